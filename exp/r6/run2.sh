#!/bin/bash
# gs_net from C++, config 5's 8-shard layout to termination, config 4's multi-GPU shapes; shard kernel A/B; 64-lane blocks A/B
set -e
O=gpurun_out/r6_run2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_dense_check.py -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -n 3 $O/tests.log
bash exp/r6/shard_ab.sh blk 2
timeout -k 10 600 python exp/ab.py --out $O/ab64 --reps 3 --variant "b128:dir=." --variant "b64:lib=safe_gossip_amd/lib_blk64.so" > $O/ab64.log 2>&1
tail -n 2 $O/ab64.log
