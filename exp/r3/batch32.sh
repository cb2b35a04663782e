#!/bin/bash
# Round 3 (session 2): (1) no event records/waits on the engine stream unless
# a side-stream build needs them, (2) per-part tail regions in the gather-path
# sort, (3) the small DLV sort's target loads issued with its region loads,
# (4) 16-byte loads for a gathered row's planes at 32 and 64 rumors.
# Full GPU suite, then A/B interleaved: new / cls3 (all but 4,
# exp/lib_cls3.so) / base (1 only, exp/lib_b31_base.so) / prev (none,
# exp/lib_prev_events.so).
set -o pipefail
OUT=gpurun_out/r3_batch32
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run() {  # variant config iteration
  L=""
  [ $1 = cls3 ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_cls3.so"
  [ $1 = base ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_b31_base.so"
  [ $1 = prev ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_prev_events.so"
  env $L timeout -k 10 300 python -u bench.py --config $2 --no-cpu-baseline --no-spread > $OUT/bench_$2_$1_$3.json 2> $OUT/bench_$2_$1_$3.err || { tail -5 $OUT/bench_$2_$1_$3.err; return 1; }
  echo "$1 $2 $(tail -1 $OUT/bench_$2_$1_$3.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
}
for it in 1 2; do
  for V in new base prev; do run $V cfg2 $it || exit 1; done
  for V in new cls3 base prev; do run $V cfg3 $it || exit 1; done
done
for V in new base prev; do for C in cfg4 cfg5; do run $V $C 1 || exit 1; done; done
for it in 1 2; do for V in new cls3; do  # the slice shape of 8 GPUs (32-bit lanes)
  L=""; [ $V = cls3 ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_cls3.so"
  env $L timeout -k 10 300 python -u bench.py --rumors 32 --no-cpu-baseline --no-spread > $OUT/bench_R32_${V}_$it.json 2> $OUT/bench_R32_${V}_$it.err || exit 1
  echo "$V R32 $(tail -1 $OUT/bench_R32_${V}_$it.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done; done
echo done
