#!/bin/bash
# HEAD validation: the whole -m gpu suite, smoke, the bench lines of configs 2-5, then rocprof kernel trace + PMC of configs 4 and 5
set -e
O=gpurun_out/r4final8; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=25 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg4.json 2> $O/bench.err
for c in cfg5 cfg2 cfg3; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err; done
bash profiles/rocprof_r2.sh r4m_cfg4
bash profiles/rocprof_r2.sh r4m_cfg5 --config cfg5
