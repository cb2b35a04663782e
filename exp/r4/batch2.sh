#!/bin/bash
# code-row shards + full-size dense checks + one RCCL rank at config 5
set -e
mkdir -p gpurun_out/r4b2
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py -k "code_rows or class_rows or (parity and not larger)" > gpurun_out/r4b2/tests_shard.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded_dist.py > gpurun_out/r4b2/tests_dist.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_verify.py > gpurun_out/r4b2/tests_dense.log 2>&1
timeout -k 10 300 python bench.py --config cfg5 --sharded --no-spread > gpurun_out/r4b2/cfg5_shard1.json 2> gpurun_out/r4b2/cfg5_shard1.err
