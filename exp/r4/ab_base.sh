#!/bin/bash
# interleaved A/B on one box: round-3 tree (_abbase) against HEAD, configs 5 and 2; kernel stats of both at config 5; shard tests
set -e
O=gpurun_out/r4ab; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sharded.py -k "code_rows or class_rows or 16 or 4 or 3" > $O/tests_shard.log 2>&1
for i in 1 2 3; do
  (cd $R/_abbase && timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread) > $O/cfg5_base_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_head_$i.json 2>>$O/err.log
  (cd $R/_abbase && timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread) > $O/cfg2_base_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_head_$i.json 2>>$O/err.log
done
cd /tmp && export TMPDIR=/tmp
cd $R/_abbase && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_base -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_head -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
