#!/bin/bash
# Whole -m gpu suite + smoke on the GPU box.  Usage: validate.sh <tag> [pytest -k expr]
set -e
T=${1:-v}; K=${2:-}
O=gpurun_out/r5v_$T; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --durations=15 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=25 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/gpu_tests.log
