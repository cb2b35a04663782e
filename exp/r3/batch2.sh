#!/bin/bash
# Round 3 batch: full-size tests to termination, bench with both multi-GPU
# modes over gloo on one GPU, the deferred RCCL slice test, then the pipe A/B.
set -o pipefail
OUT=gpurun_out/r3_batch2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_cfg5.py -v -s --timeout 500 --timeout-method thread > $OUT/fullsize.log 2>&1 || { tail -40 $OUT/fullsize.log; exit 1; }
grep -E "spread n=|passed|failed" $OUT/fullsize.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_sliced.py tests/test_gpu_api.py tests/test_gpu_wire.py -q --timeout 250 --timeout-method thread > $OUT/sliced_api.log 2>&1 || { tail -40 $OUT/sliced_api.log; exit 1; }
tail -1 $OUT/sliced_api.log
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --nodes 1048576 --steps 6 --warmup 2 --no-spread > $OUT/bench_gloo2_cfg4small.json 2> $OUT/bench_gloo2_cfg4small.err || { tail -20 $OUT/bench_gloo2_cfg4small.err; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --config cfg5 --nodes 4000000 --steps 6 --warmup 2 --no-spread > $OUT/bench_gloo2_cfg5small.json 2> $OUT/bench_gloo2_cfg5small.err || { tail -20 $OUT/bench_gloo2_cfg5small.err; exit 1; }
timeout -k 10 300 python -u bench.py --sharded --no-cpu-baseline --no-spread > $OUT/bench_sharded1.json 2> $OUT/bench_sharded1.err || { tail -20 $OUT/bench_sharded1.err; exit 1; }
bash exp/r3/ab_pipe2.sh
