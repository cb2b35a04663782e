#!/bin/bash
# code-row shards: parity (local shards, gloo, one RCCL rank), then one RCCL rank at config 5
set -e
mkdir -p gpurun_out/r4sd
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py -k "code_rows or class_rows or dist or (parity and (16 or 4 or 3 or 7 or 1))" > gpurun_out/r4sd/tests.log 2>&1
timeout -k 10 300 python bench.py --config cfg5 --sharded --no-spread > gpurun_out/r4sd/cfg5_shard1.json 2> gpurun_out/r4sd/cfg5_shard1.err
timeout -k 10 300 python bench.py --config cfg5 --sharded --parts 1 --no-spread > gpurun_out/r4sd/cfg5_shard1_p1.json 2>> gpurun_out/r4sd/cfg5_shard1.err
