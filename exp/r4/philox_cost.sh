#!/bin/bash
# config 5's build kernels with 3 / 2 / 1 Philox draws per source in dl_coarse (faults with churn / without churn / none)
set -e
O=gpurun_out/r4philox; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/full -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/full.json 2>>$O/err.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/nochurn -o run -- python3 bench.py --config cfg5 --churn 0 --no-cpu-baseline --no-spread > $O/nochurn.json 2>>$O/err.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/none -o run -- python3 bench.py --config cfg5 --churn 0 --drop-push 0 --drop-pull 0 --no-cpu-baseline --no-spread > $O/none.json 2>>$O/err.log
