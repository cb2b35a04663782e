#!/bin/bash
# Kernel-trace + stats profile of a bench workload, then separate PMC passes
# (one counter group per run, as MI355X_MICROARCH.md prescribes).
# Run on the GPU box from the repo root:
#   bash profiles/rocprof_r2.sh <tag> [bench args...]
set -e
TAG=${1:-r2}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# the bench default window (20 timed rounds from injection, 3 warmup rounds)
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-spread $*"
# (the PMC passes run the bench without its own live PMC children: a profiled
# process may not start a second profiler)
PARGS="$ARGS --pmc off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ROOT/bench.py $PARGS > $OUT/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ROOT/bench.py $PARGS > $OUT/write.log 2>&1
echo done
