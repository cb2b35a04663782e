#!/bin/bash
# Round 3: zero-over-zero store skip + LDS swizzle in round_kernel, interleaved
# A/B on one box (base = neither, noz = swizzle only, head = both), after the
# parity suite of the wide 2P path.
set -o pipefail
OUT=gpurun_out/r3_zskip
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for i in 1 2 3; do
for V in base noz head; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/bench_${V}_$i.json 2> $OUT/bench_${V}_$i.err || exit 1
done
done
echo done
