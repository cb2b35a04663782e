#!/bin/bash
# kernel trace of one RCCL rank at config 5 (code-row shards)
set -e
O=gpurun_out/r4ps5; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config cfg5 --sharded --no-spread --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python -u -m pytest -x -v --durations=0 --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py > $O/tests_dense.log 2>&1
