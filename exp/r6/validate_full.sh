#!/bin/bash
# Round-6 validation of the tree: whole -m gpu suite, smoke, 8-shard kernel A/B
# against exp/base_tree, the default bench line (live PMC), config 5's line,
# and the rocprofv3 kernel-trace + PMC passes of config 4.  Usage: validate_full.sh <tag>
set -e
T=${1:-v}
O=gpurun_out/r6v_$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -n 2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > $O/bench_cfg4.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2>> $O/bench.err
bash profiles/rocprof_r2.sh ${T}_cfg4
bash exp/r6/shard_ab.sh $T 1
