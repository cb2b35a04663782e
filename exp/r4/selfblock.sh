#!/bin/bash
# code-row shards: rows and pulls of a rank's own block written straight into its receive buffers (one rank exchanges nothing)
set -e
O=gpurun_out/r4self; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py > $O/tests_shard.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py -k "config5" > $O/tests_cfg5.log 2>&1
for i in 1 2; do
  (cd $R/_abbase && timeout -k 10 300 python bench.py --config cfg5 --sharded --no-cpu-baseline --no-spread) > $O/shard1_base_$i.json 2>>$O/err.log
  timeout -k 10 300 python bench.py --config cfg5 --sharded --no-cpu-baseline --no-spread > $O/shard1_head_$i.json 2>>$O/err.log
done
