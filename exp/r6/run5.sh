#!/bin/bash
# bench.py's library-loop modes on one RCCL rank (config 4 and 5), the Python
# drivers beside them, and the watchdog rehearsed with two gloo ranks
set -e
O=gpurun_out/r6_run5; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in nodes-lib slices-lib nodes slices; do
  timeout -k 10 300 python bench.py --sharded --mode $m --no-spread --pmc off >> $O/cfg4_w1.jsonl 2>> $O/err.log
done
for m in nodes-lib nodes; do
  timeout -k 10 300 python bench.py --config cfg5 --sharded --mode $m --no-spread --pmc off >> $O/cfg5_w1.jsonl 2>> $O/err.log
done
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --deadline 40 > $O/gloo2_watchdog.jsonl 2>> $O/err.log
grep -h '^{' $O/*.jsonl | cut -c1-300
