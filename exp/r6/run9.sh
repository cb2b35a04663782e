#!/bin/bash
set -e
O=gpurun_out/r6_run9; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
bash exp/r6/shard_ab.sh pf 2
