#!/bin/bash
# Round 3: (1) Philox products as v_mad_u64_u32 (microbenchmark), (2) the DLV
# build reads the round kernel's fault bits (parity + an interleaved cfg5 A/B:
# a = r2 draws, b = 64-bit products only, head = both), (3) the single-part
# stall fixed (chunked RCCL exchanges), (4) traces of the small configs,
# (5) 8K-target bins (lib_bin13: one sort block per bin, no half split).
set -o pipefail
OUT=gpurun_out/r3_batch7
mkdir -p $OUT
timeout -k 10 60 ./exp/r3/philox_mb > $OUT/philox_mb.log 2>&1 || { cat $OUT/philox_mb.log; exit 1; }
cat $OUT/philox_mb.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg5.py -x -q --timeout 200 --timeout-method thread -k "faults or delivery or config5 or seq" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_bin13.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "delivery or faults" > $OUT/parity_bin13.log 2>&1 || { tail -30 $OUT/parity_bin13.log; exit 1; }
tail -2 $OUT/parity_bin13.log
for i in 1 2; do
for V in r3a r3b head bin13; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "$V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
done
for V in head bin13; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/cfg4_${V}.json 2> $OUT/cfg4_${V}.err || exit 1
  echo "cfg4 $V $(tail -1 $OUT/cfg4_${V}.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_dist.py -v --timeout 300 --timeout-method thread > $OUT/sharded_dist.log 2>&1 || { tail -40 $OUT/sharded_dist.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/sharded_dist.log | tail -8
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg3; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_$C.log 2>&1 || exit 1
done
echo done
