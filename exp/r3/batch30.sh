#!/bin/bash
# Round 3 (session 2): no event records/waits on the engine stream unless a
# side-stream build needs them.  Full GPU suite, then A/B against the
# previous engine (exp/lib_prev_events.so), interleaved, configs 2-5.
set -o pipefail
OUT=gpurun_out/r3_batch30
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for it in 1 2; do
  for V in new prev; do
    L=""; [ $V = prev ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_prev_events.so"
    for C in cfg2 cfg3 cfg4 cfg5; do
      env $L timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/bench_${C}_${V}_$it.json 2> $OUT/bench_${C}_${V}_$it.err || { tail -5 $OUT/bench_${C}_${V}_$it.err; exit 1; }
      echo "$V $C $(tail -1 $OUT/bench_${C}_${V}_$it.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
    done
  done
done
echo done
