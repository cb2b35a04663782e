#!/bin/bash
# Round 3 (session 2): quarter-bin DLV sorts as the default at n >= 2^21;
# config-5 A/B of the coarse bucket width (64 / 128 / 256 bins); GPU suite.
set -o pipefail
OUT=gpurun_out/r3_batch15
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for V in cb64 cb256; do
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_$V.so timeout -k 10 300 $T tests/test_gpu_fullsize.py -m gpu -k "partition" > $OUT/tests_$V.log 2>&1 || { tail -30 $OUT/tests_$V.log; exit 1; }
tail -1 $OUT/tests_$V.log
done
for i in 1 2; do
for V in head cb64 cb256; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for C in cfg2 cfg3; do
  timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}.json 2> $OUT/${C}.err || exit 1
  echo "$C $(tail -1 $OUT/${C}.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
echo done
