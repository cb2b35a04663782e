#!/bin/bash
# Round 3: round_kernel vs the pipelined kernel with a plane-major (pm) or a
# node-major swizzled (nm) LDS image, interleaved on one box.
set -o pipefail
OUT=gpurun_out/r3_pipe2
mkdir -p $OUT
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_pipenm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "pipe" > $OUT/parity_nm.log 2>&1 || { tail -30 $OUT/parity_nm.log; exit 1; }
tail -1 $OUT/parity_nm.log
for i in 1 2 3; do
  SAFE_GOSSIP_AMD_LIB=exp/r3/lib_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/bench_rk_$i.json 2> $OUT/e || exit 1
  SAFE_GOSSIP_AMD_PIPE=1 SAFE_GOSSIP_AMD_LIB=exp/r3/lib_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/bench_pm_$i.json 2> $OUT/e || exit 1
  SAFE_GOSSIP_AMD_PIPE=1 SAFE_GOSSIP_AMD_LIB=exp/r3/lib_pipenm.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/bench_nm_$i.json 2> $OUT/e || exit 1
done
echo done
