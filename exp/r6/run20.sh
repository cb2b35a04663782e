#!/bin/bash
# Per-rank kernels of config 4's 8-GPU node-shard shape at HEAD (8 local
# shards on one GPU, kernels serialised, 30 rounds after 1)
set -e
O=gpurun_out/r6_run20; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/head -o run -- python3 exp/shard_prof.py 8 30 1 > $O/head.txt 2>&1
echo done
