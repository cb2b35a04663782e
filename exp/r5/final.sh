#!/bin/bash
# HEAD validation: the whole -m gpu suite, smoke, the default bench line (live PMC) and config 5's
set -e
T=${1:-f}
O=gpurun_out/r5final_$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > $O/bench_cfg4.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2>> $O/bench.err
tail -n 2 $O/gpu_tests.log
