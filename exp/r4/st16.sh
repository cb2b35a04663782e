#!/bin/bash
# u16 Statistics deltas on the delivery-record engines: parity, then interleaved A/B (u32 via SAFE_GOSSIP_AMD_STATS32=1)
set -e
O=gpurun_out/r4st16; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wire.py tests/test_gpu_sliced.py tests/test_gpu_sharded.py tests/test_gpu_api.py tests/test_gpu_harness.py > $O/tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py -k "config5 or small" tests/test_gpu_cfg5.py > $O/tests_cfg5.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_st16_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_STATS32=1 timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_st32_$i.json 2>>$O/err.log
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_st16_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_STATS32=1 timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_st32_$i.json 2>>$O/err.log
done
