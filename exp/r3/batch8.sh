#!/bin/bash
# Round 3: small-network builds (parts written straight into the sort blocks'
# regions, DLV pulls written directly) -- parity, cfg2/cfg3 A/B against
# lib_base (round-3 start); per-kernel cfg5 traces with and without the fault
# bits (head vs lib_r3b); cfg5 A/B of per-part regions (head vs lib_binreg).
set -o pipefail
OUT=gpurun_out/r3_batch8
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_wire.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for i in 1 2; do
for C in cfg2 cfg3; do
for V in base head; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}_${V}_$i.json 2> $OUT/${C}_${V}_$i.err || exit 1
  echo "$C $V $i $(tail -1 $OUT/${C}_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
done
done
for i in 1 2; do
for V in r3b binreg head; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
done
cd /tmp && export TMPDIR=/tmp
for V in head r3b; do
  if [ $V = head ]; then L=$GRAFT_REPO_ROOT/safe_gossip_amd/libsafe_gossip_amd.so; else L=$GRAFT_REPO_ROOT/exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_cfg5_$V -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 10 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_cfg5_$V.log 2>&1 || exit 1
done
for C in cfg2 cfg3; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_$C.log 2>&1 || exit 1
done
echo done
