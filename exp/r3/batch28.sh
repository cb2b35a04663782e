#!/bin/bash
# Round 3 (session 2): kernel traces of configs 2 and 3 at HEAD (per-step
# kernel sum vs gaps between kernels).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r3_batch28
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$C -o run -- python3 $ROOT/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-spread > $OUT/trace_$C.log 2>&1 || { tail -5 $OUT/trace_$C.log; exit 1; }
  echo $C traced
done
echo done
