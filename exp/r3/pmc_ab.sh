#!/bin/bash
# Round 3: per-dispatch HBM traffic (FETCH_SIZE, WRITE_SIZE) and kernel trace
# of the cfg4 bench window, pipelined kernel vs round_kernel.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r3_pmc_ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-spread"
for V in pipe nopipe; do
  if [ $V = nopipe ]; then export SAFE_GOSSIP_AMD_PIPE=0; else unset SAFE_GOSSIP_AMD_PIPE; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V/trace -o run -- python3 $ROOT/bench.py $ARGS > $OUT/$V.trace.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$V/fetch -o run -- python3 $ROOT/bench.py $ARGS > $OUT/$V.fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$V/write -o run -- python3 $ROOT/bench.py $ARGS > $OUT/$V.write.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/$V/sq -o run -- python3 $ROOT/bench.py $ARGS > $OUT/$V.sq.log 2>&1 || exit 1
done
echo done
