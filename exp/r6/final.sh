#!/bin/bash
# Round-6 HEAD validation: the whole -m gpu suite, smoke, bench lines of
# configs 4 (live PMC, CPU baselines), 5, 2 and 3, rocprofv3 kernel-trace +
# PMC passes of configs 4 and 5.  Usage: final.sh <tag>
# (bench.py --gpus 8 rehearsed with 8 gloo ranks: exp/r6/rehearse8.sh)
set -e
T=${1:-f}
O=gpurun_out/r6final_$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=25 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -n 2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > $O/bench_cfg4.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2>> $O/bench.err
for c in cfg2 cfg3; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --pmc off > $O/bench_$c.json 2>> $O/bench.err; done
bash profiles/rocprof_r2.sh ${T}_cfg4
bash profiles/rocprof_r2.sh ${T}_cfg5 --config cfg5
