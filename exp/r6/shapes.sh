#!/bin/bash
# Per-rank shapes of the driver's N = 2, 4, 8 runs on one GPU: rumor slices of
# config 4 (2^24 x 256/N) as bench lines, and config 5's 8 code-row shards
# (kernels serialised under rocprofv3).  Usage: shapes.sh <tag>
set -e
T=${1:-s}
O=gpurun_out/r6shape_$T; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
for r in 128 64 32; do
  timeout -k 10 200 python bench.py --rumors $r --no-cpu-baseline --no-spread --pmc off > $O/slice_R$r.json 2>> $O/err.log
done
PARTS=4 AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/shard8_cfg5 -o run -- python3 exp/shard_prof.py 8 20 3 cfg5 > $O/shard8_cfg5.txt 2>&1
PARTS=4 timeout -k 10 200 python3 exp/shard_prof.py 8 20 3 > $O/shard8_cfg4_wall.txt 2>&1
grep -h ms_per_step $O/slice_R*.json | cut -c1-10 >/dev/null || true
