#!/bin/bash
# Round 3: first GPU run of the pipelined round kernel (gs_pipe.hip).
set -o pipefail
OUT=gpurun_out/r3_pipe1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "pipe or round_kernel_wide" > $OUT/pipe_tests.log 2>&1 || { tail -30 $OUT/pipe_tests.log; exit 1; }
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/bench_pipe_$i.json 2> $OUT/bench_pipe_$i.err || exit 1
SAFE_GOSSIP_AMD_PIPE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-spread > $OUT/bench_nopipe_$i.json 2> $OUT/bench_nopipe_$i.err || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
