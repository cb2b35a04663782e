#!/bin/bash
# Per-rank cost of config 4's 8-GPU shapes on one GPU: 8 local node shards
# (serialised kernel trace + concurrent wall time), and one rumor slice
# (2^24 x 32) -- bench line + kernel trace.  Usage: mgpu_prof.sh <tag>
set -e
T=${1:-base}
O=gpurun_out/r5mg_$T; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 python3 exp/shard_prof.py 8 30 1 > $O/shard8_wall.txt 2>&1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/shard8 -o run -- python3 exp/shard_prof.py 8 30 1 > $O/shard8_ser.txt 2>&1
timeout -k 10 200 python3 bench.py --rumors 32 --steps 30 --warmup 3 --no-cpu-baseline --no-spread > $O/slice32.json 2>$O/slice32.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/slice32 -o run -- python3 bench.py --rumors 32 --steps 30 --warmup 3 --no-cpu-baseline --no-spread > /dev/null 2>>$O/slice32.err
