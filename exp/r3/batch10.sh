#!/bin/bash
# Round 3 (session 2): coarse-bucket fill shards for the DLV build (A/B at
# config 5: 1 / 4 / 8 shards), the new DLV-vs-gather build test, host enqueue
# cost of small networks, and a config-4 kernel trace at HEAD.
set -o pipefail
OUT=gpurun_out/r3_batch10
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_fullsize.py -k "dlv" -m gpu > $OUT/tests_head.log 2>&1 || { tail -30 $OUT/tests_head.log; exit 1; }
tail -1 $OUT/tests_head.log
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_sh4.so timeout -k 10 300 $T tests/test_gpu_fullsize.py -k "partition" -m gpu > $OUT/tests_sh4.log 2>&1 || { tail -30 $OUT/tests_sh4.log; exit 1; }
tail -1 $OUT/tests_sh4.log
for i in 1 2; do
for V in head sh4 sh8; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
timeout -k 10 200 python -u exp/r3/host_overhead.py > $OUT/host_overhead.jsonl 2> $OUT/host_overhead.err || exit 1
cat $OUT/host_overhead.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_cfg4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_cfg4.log 2>&1 || exit 1
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/exp/r3/lib_sh4.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_cfg5_sh4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_cfg5_sh4.log 2>&1 || exit 1
echo done
