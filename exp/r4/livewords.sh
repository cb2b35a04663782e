#!/bin/bash
# the any-live flag as plain stores into 64 strided words (no read at a block's end): parity, then interleaved A/B against the previous commit (_abbase)
set -e
O=gpurun_out/r4live; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wire.py tests/test_gpu_sliced.py tests/test_gpu_sharded.py tests/test_gpu_api.py tests/test_gpu_harness.py > $O/tests.log 2>&1
for i in 1 2 3; do
  for c in cfg4 cfg5 cfg3; do
    (cd $R/_abbase && timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-spread) > $O/${c}_base_$i.json 2>>$O/err.log
    timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-spread > $O/${c}_head_$i.json 2>>$O/err.log
  done
done
cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_cfg4 -o run -- python3 bench.py --config cfg4 --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
