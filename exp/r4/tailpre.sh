#!/bin/bash
# the DLV round kernel loads the first tail codes of every node with its metadata: parity, then interleaved A/B
# base = previous commit (_abbase), pre1 = one tail code per node (GS_DLV4_TAIL_PRE=1), head = two
set -e
O=gpurun_out/r4pre; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wire.py tests/test_gpu_sliced.py tests/test_gpu_sharded.py tests/test_gpu_api.py tests/test_gpu_harness.py > $O/tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py -k "config5 or small" tests/test_gpu_cfg5.py > $O/tests_cfg5.log 2>&1
for i in 1 2 3; do
  (cd $R/_abbase && timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread) > $O/cfg5_base_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pre1.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_pre1_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_head_$i.json 2>>$O/err.log
  (cd $R/_abbase && timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread) > $O/cfg2_base_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_head_$i.json 2>>$O/err.log
done
cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_head -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pre1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_pre1 -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
