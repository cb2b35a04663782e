#!/bin/bash
# Round 3 (session 2): (1) no event records/waits on the engine stream unless
# a side-stream build needs them, (2) per-part tail regions in the gather-path
# sort, (3) the small DLV sort's target loads issued with its region loads.
# Full GPU suite, then A/B interleaved: new / base (1 only,
# exp/lib_b31_base.so) / prev (none, exp/lib_prev_events.so).
set -o pipefail
OUT=gpurun_out/r3_batch31
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run() {  # variant config iteration
  L=""; [ $1 = base ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_b31_base.so"; [ $1 = prev ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_prev_events.so"
  env $L timeout -k 10 300 python -u bench.py --config $2 --no-cpu-baseline --no-spread > $OUT/bench_$2_$1_$3.json 2> $OUT/bench_$2_$1_$3.err || { tail -5 $OUT/bench_$2_$1_$3.err; return 1; }
  echo "$1 $2 $(tail -1 $OUT/bench_$2_$1_$3.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
}
for it in 1 2; do for V in new base prev; do for C in cfg2 cfg3; do run $V $C $it || exit 1; done; done; done
for V in new base prev; do for C in cfg4 cfg5; do run $V $C 1 || exit 1; done; done
echo done
