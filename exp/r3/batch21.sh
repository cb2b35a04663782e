#!/bin/bash
# Round 3 (session 2): the config-5 transition kernel forced to 8 waves per
# SIMD (GS_DLV4_MINW=8, 9 VGPRs spilled) and the gather path with 8 sort
# blocks per bin below 2^21 nodes (config 3): parity first, then A/B.
set -o pipefail
OUT=gpurun_out/r3_batch21
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_small.so timeout -k 10 600 $T tests/test_gpu_parity.py -m gpu > $OUT/tests_small.log 2>&1 || { tail -5 $OUT/tests_small.log; exit 1; }
tail -1 $OUT/tests_small.log
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_dlv8.so timeout -k 10 600 $T tests/test_gpu_fullsize.py -m gpu -k "dlv" > $OUT/tests_dlv8.log 2>&1 || { tail -5 $OUT/tests_dlv8.log; exit 1; }
tail -1 $OUT/tests_dlv8.log
for i in 1 2 3; do
for V in head dlv8; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
for V in head small; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg3 --no-cpu-baseline --no-spread > $OUT/cfg3_${V}_$i.json 2> $OUT/cfg3_${V}_$i.err || exit 1
  echo "cfg3 $V $i $(tail -1 $OUT/cfg3_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
echo done
