#!/bin/bash
# Round 3 (session 2): dl_fine with 8 K-entry chunks (half the reservation
# atomics): parity at the config-5 shape and config-5 A/B; the failing call of
# the small-network split variant.
set -o pipefail
OUT=gpurun_out/r3_batch18
mkdir -p $OUT
SAFE_GOSSIP_AMD_DEBUG=1 SAFE_GOSSIP_AMD_LIB=exp/r3/lib_small.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "example" --timeout 100 --timeout-method thread > $OUT/tests_small.log 2>&1; grep -a "safe_gossip_amd:" $OUT/tests_small.log | head -3; tail -1 $OUT/tests_small.log
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_fc8k.so timeout -k 10 300 $T tests/test_gpu_fullsize.py -m gpu -k "partition" > $OUT/tests_fc8k.log 2>&1 || { tail -30 $OUT/tests_fc8k.log; exit 1; }
tail -1 $OUT/tests_fc8k.log
for i in 1 2 3; do
for V in head fc8k; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
cd /tmp && export TMPDIR=/tmp
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/exp/r3/lib_fc8k.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_fc8k -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_fc8k.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_head -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_head.log 2>&1 || exit 1
echo done
