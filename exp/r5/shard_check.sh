#!/bin/bash
# shard tests + the 8-GPU shapes' dense check + the shape profile
set -e
T=${1:-d}
O=gpurun_out/r5sc_$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense_check.py -m gpu -x -q -k "multi_gpu" --timeout 300 --timeout-method thread >> $O/tests.log 2>&1
bash exp/r5/mgpu_prof.sh $T
tail -2 $O/tests.log
