#!/bin/bash
# DLV flag bytes + the mutual bit in the pushers' source field instead of 4-B target words: parity incl. shards and the fused partition, then interleaved A/B
set -e
O=gpurun_out/r4fl; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wire.py tests/test_gpu_sliced.py tests/test_gpu_sharded.py tests/test_gpu_api.py tests/test_gpu_harness.py tests/test_gpu_sharded_dist.py > $O/tests.log 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_cfg5.py tests/test_gpu_fullsize.py -k "config5 or small or partition or packed" > $O/tests_cfg5.log 2>&1
for i in 1 2 3; do
  (cd $R/_abbase && timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread) > $O/cfg5_base_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_head_$i.json 2>>$O/err.log
  (cd $R/_abbase && timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread) > $O/cfg2_base_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_head_$i.json 2>>$O/err.log
done
cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_head -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
