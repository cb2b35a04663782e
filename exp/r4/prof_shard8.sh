#!/bin/bash
# per-shard kernel times: 8 local shards of config 5 (and of config 4), kernels serialised
set -e
O=gpurun_out/r4ps8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg5 -o run -- python3 exp/shard_prof.py 8 8 3 cfg5 > $O/cfg5.txt 2>&1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg4 -o run -- python3 exp/shard_prof.py 8 8 3 > $O/cfg4.txt 2>&1
