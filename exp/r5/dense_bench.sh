#!/bin/bash
# the full-size dense checks, then the default bench line (live PMC traffic)
set -e
O=gpurun_out/r5db_${1:-a}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_dense_check.py -x -v --durations=10 --timeout 500 --timeout-method thread > $O/dense.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
tail -3 $O/dense.log
