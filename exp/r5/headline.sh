#!/bin/bash
# bench lines (default = config 4, with live PMC traffic; configs 5, 2, 3) and
# the rocprofv3 kernel-trace + PMC passes of configs 4 and 5.  Usage: headline.sh <tag>
set -e
T=${1:-h}
O=gpurun_out/r5h_$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > $O/bench_cfg4.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2>> $O/bench.err
for c in cfg2 cfg3; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --pmc off > $O/bench_$c.json 2>> $O/bench.err; done
bash profiles/rocprof_r2.sh ${T}_cfg4
bash profiles/rocprof_r2.sh ${T}_cfg5 --config cfg5
