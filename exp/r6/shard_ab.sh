#!/bin/bash
# Per-rank kernels of config 4's 8-GPU node-shard shape (8 local shards on one
# GPU, kernels serialised, 30 rounds after 1) for the tree and exp/base_tree,
# interleaved.  Usage: shard_ab.sh <tag> [reps]
set -e
T=${1:-s}; N=${2:-2}
O=gpurun_out/r6sh_$T; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
for i in $(seq 1 $N); do
  for v in base head; do
    d=$R; [ $v = base ] && d=$R/exp/base_tree
    GS_TREE=$d AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/${v}_$i -o run -- python3 exp/shard_prof.py 8 30 1 > $O/${v}_$i.txt 2>&1
  done
done
