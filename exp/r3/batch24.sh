#!/bin/bash
# Round 3 (session 2): config-4 round kernel with the b planes read late from
# the stage (103 VGPRs), and with the Statistics loaded late too at 5 waves
# per SIMD (96 VGPRs, 3 spilled): parity of the latter, then A/B; also
# inl_sort on half bins with 512-thread blocks (two per CU).
set -o pipefail
OUT=gpurun_out/r3_batch24
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_lb5.so timeout -k 10 600 $T tests/test_gpu_parity.py -m gpu -k "round_parity or filtered or wide or unfiltered or faults" > $OUT/tests_lb5.log 2>&1 || { tail -30 $OUT/tests_lb5.log; exit 1; }
tail -1 $OUT/tests_lb5.log
for i in 1 2 3; do
for V in head lb lb5 s512; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/cfg4_${V}_$i.json 2> $OUT/cfg4_${V}_$i.err || exit 1
  echo "cfg4 $V $i $(tail -1 $OUT/cfg4_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
echo done
