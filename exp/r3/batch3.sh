#!/bin/bash
# Round 3 batch: API test fix, bench with both multi-GPU modes over gloo on one
# GPU, the single-part RCCL shape, then the pipe A/B.
set -o pipefail
OUT=gpurun_out/r3_batch3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_verify.py -q --timeout 250 --timeout-method thread > $OUT/api.log 2>&1 || { tail -40 $OUT/api.log; exit 1; }
tail -1 $OUT/api.log
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --nodes 1048576 --steps 6 --warmup 2 --no-spread > $OUT/bench_gloo2_cfg4small.json 2> $OUT/bench_gloo2_cfg4small.err || { tail -20 $OUT/bench_gloo2_cfg4small.err; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --config cfg5 --nodes 4000000 --steps 6 --warmup 2 --no-spread > $OUT/bench_gloo2_cfg5small.json 2> $OUT/bench_gloo2_cfg5small.err || { tail -20 $OUT/bench_gloo2_cfg5small.err; exit 1; }
timeout -k 10 300 python -u bench.py --sharded --no-cpu-baseline --no-spread > $OUT/bench_sharded1.json 2> $OUT/bench_sharded1.err || { tail -20 $OUT/bench_sharded1.err; exit 1; }
NCCL_DEBUG=WARN timeout -k 10 180 python -u exp/r3/rccl_p1.py 24 1 256 > $OUT/rccl_p1.log 2>&1; echo "rccl_p1 rc=$?"; tail -5 $OUT/rccl_p1.log
bash exp/r3/ab_pipe2.sh
