#!/bin/bash
# Round 3: the whole GPU suite after the build changes (per-part regions, the
# small-network DLV build, counters cleared by the round kernel, Philox
# products as v_mad_u64_u32), then the bench configs and their traces; cfg5
# A/B of the Philox products (head vs lib_mulhi).
set -o pipefail
OUT=gpurun_out/r3_batch9
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for i in 1 2; do
for C in cfg2 cfg3; do
  timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}_$i.json 2> $OUT/${C}_$i.err || exit 1
  echo "$C $i $(tail -1 $OUT/${C}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
for V in mulhi head; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/cfg4.json 2> $OUT/cfg4.err || exit 1
echo "cfg4 $(tail -1 $OUT/cfg4.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg3 cfg5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_$C.log 2>&1 || exit 1
done
echo done
