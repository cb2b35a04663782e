#!/bin/bash
# Round 3 (session 2) final HEAD validation: the GPU suite, smoke, every bench
# config, rocprof kernel traces and HBM (FETCH/WRITE) passes of configs 4
# and 5; then the gather path with 8 sort blocks per bin below 2^21 nodes
# (parity first, config 3 A/B).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r3_head3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || exit 1
tail -1 $OUT/bench_cfg4.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("cfg4", d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["cpu_baseline"]["value"], d["spread"])'
for C in cfg2 cfg3 cfg5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || exit 1
  echo "$C $(tail -1 $OUT/bench_$C.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["spread"])')"
done
timeout -k 10 300 python -u bench.py --rumors 32 --no-cpu-baseline --no-spread > $OUT/bench_cfg4_R32.json 2> $OUT/bench_cfg4_R32.err || exit 1
echo "2^24x32 $(tail -1 $OUT/bench_cfg4_R32.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"][:24])')"
timeout -k 10 700 bash profiles/rocprof_r2.sh r3_head3_cfg4 > $OUT/prof_cfg4.log 2>&1 || { tail -5 $OUT/prof_cfg4.log; exit 1; }
timeout -k 10 700 bash profiles/rocprof_r2.sh r3_head3_cfg5 --config cfg5 > $OUT/prof_cfg5.log 2>&1 || { tail -5 $OUT/prof_cfg5.log; exit 1; }
echo profiles done
# A/B: the two-phase build (inl_bin beside the round kernel) at config 3
for it in 1 2; do for S in 0 1; do
  SAFE_GOSSIP_AMD_SPLIT_BUILD=$S timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline --no-spread > $OUT/ab_cfg3_split${S}_$it.json 2> $OUT/ab_cfg3_split${S}_$it.err || exit 1
  echo "split=$S cfg3 $(tail -1 $OUT/ab_cfg3_split${S}_$it.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done; done
echo done
