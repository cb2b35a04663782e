#!/bin/bash
# Round 3: the single-part stall fixed (chunked RCCL exchanges), sharded dist
# tests; kernel traces of the small configs (where does a cfg2/cfg3 step go?)
set -o pipefail
OUT=gpurun_out/r3_batch6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_dist.py -v --timeout 300 --timeout-method thread > $OUT/sharded_dist.log 2>&1 || { tail -40 $OUT/sharded_dist.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/sharded_dist.log | tail -8
timeout -k 10 200 python -u exp/r3/rccl_p1.py 24 1 256 nccl > $OUT/p1_fixed.log 2>&1; echo "p1 fixed rc=$?"; grep -v "WARN\|^$" $OUT/p1_fixed.log | tail -4
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg3; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_$C.log 2>&1 || exit 1
done
echo done
