#!/bin/bash
# Round 3 (session 2): the 32-bit lane round kernel (gs_w32.hip): parity,
# full-size equivalence with the 64-bit lane kernel, config-4 A/B (w32 /
# w32 at 8 waves / w64), config-5 A/B of quarter-bin DLV sorts (two blocks
# per CU), host enqueue cost with fence-free timing events.
set -o pipefail
OUT=gpurun_out/r3_batch11
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py -m gpu -k "w32 or round_kernel_wide or filtered_larger or test_round_parity" > $OUT/tests_parity.log 2>&1 || { tail -40 $OUT/tests_parity.log; exit 1; }
tail -1 $OUT/tests_parity.log
timeout -k 10 400 $T tests/test_gpu_fullsize.py -m gpu -k "w32 or dlv" > $OUT/tests_full.log 2>&1 || { tail -40 $OUT/tests_full.log; exit 1; }
tail -1 $OUT/tests_full.log
for i in 1 2; do
for V in w32 w64 m8; do
  L=safe_gossip_amd/libsafe_gossip_amd.so; E=1
  if [ $V = w64 ]; then E=0; fi
  if [ $V = m8 ]; then L=exp/r3/lib_w32m8.so; fi
  SAFE_GOSSIP_AMD_W32=$E SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/cfg4_${V}_$i.json 2> $OUT/cfg4_${V}_$i.err || exit 1
  echo "cfg4 $V $i $(tail -1 $OUT/cfg4_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
done
for i in 1 2; do
for V in head dsl2; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
timeout -k 10 200 python -u exp/r3/host_overhead.py > $OUT/host_overhead.jsonl 2> $OUT/host_overhead.err || exit 1
cat $OUT/host_overhead.jsonl
for C in cfg2 cfg3; do
  timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}.json 2> $OUT/${C}.err || exit 1
  echo "$C $(tail -1 $OUT/${C}.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_cfg4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_cfg4.log 2>&1 || exit 1
echo done
