#!/bin/bash
# one node per 32-bit lane below R_pad 16 (SAFE_GOSSIP_AMD_DLV_PACK=u32x1): parity with it forced, then config 2 interleaved against the default (four nodes per lane)
set -e
O=gpurun_out/r4pack1; mkdir -p $O
SAFE_GOSSIP_AMD_DLV_PACK=u32x1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wire.py > $O/tests_u32x1.log 2>&1
SAFE_GOSSIP_AMD_DLV_PACK=u32x1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py -k "small" > $O/tests_dense_u32x1.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_head_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_DLV_PACK=u32x1 timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_x1_$i.json 2>>$O/err.log
done
