#!/bin/bash
# shard parity with 128-lane shard blocks, config 5 / config 4 full-size multi-GPU layouts, shard kernel A/B
set -e
O=gpurun_out/r6_run1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py tests/test_gpu_dense_check.py -m gpu -x -q --durations=10 --timeout 600 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
bash exp/r6/shard_ab.sh blk 2
