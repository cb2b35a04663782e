#!/bin/bash
# Round 3 (session 2): small networks with 8 / 16 sort blocks per bin
# (gather path inl_sort<3>, DLV quarter.. sixteenth bins): parity, then
# configs 2 and 3 A/B.
set -o pipefail
OUT=gpurun_out/r3_batch17
mkdir -p $OUT
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_small.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_small.log 2>&1 || { tail -30 $OUT/tests_small.log; exit 1; }
tail -1 $OUT/tests_small.log
for i in 1 2 3; do
for V in head small; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  for C in cfg2 cfg3; do
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}_${V}_$i.json 2> $OUT/${C}_${V}_$i.err || exit 1
  echo "$C $V $i $(tail -1 $OUT/${C}_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
done
cd /tmp && export TMPDIR=/tmp
for V in head small; do
  if [ $V = head ]; then L=$GRAFT_REPO_ROOT/safe_gossip_amd/libsafe_gossip_amd.so; else L=$GRAFT_REPO_ROOT/exp/r3/lib_$V.so; fi
  for C in cfg2 cfg3; do
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_${C}_$V -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_${C}_$V.log 2>&1 || exit 1
  done
done
echo done
