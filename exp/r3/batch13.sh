#!/bin/bash
# Round 3 (session 2): which HIP call the quarter-bin DLV variant fails at
# 10^8 nodes; the GPU suite at the current tree (w32 default at R_pad 32, DLV
# sort reading 32-bit plane halves, part index kept per partition entry).
set -o pipefail
OUT=gpurun_out/r3_batch13
mkdir -p $OUT
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_dsl2.so SAFE_GOSSIP_AMD_DEBUG=1 timeout -k 10 120 python -u exp/r3/dsl2_diag.py 100000000 > $OUT/dsl2_diag.log 2>&1; echo "dsl2 diag rc=$?"; grep -v amdgpu.ids $OUT/dsl2_diag.log | tail -4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for C in cfg5 cfg4; do
  timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}.json 2> $OUT/${C}.err || exit 1
  echo "$C $(tail -1 $OUT/${C}.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
echo done
