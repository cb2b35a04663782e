#!/bin/bash
# A kernel change checked and timed on one box: a parity subset, then
# interleaved A/B runs (exp/ab.py) of the base tree (exp/base_tree, the
# previous commit built there) against this tree on the given workloads.
#   bash exp/ab_round.sh <tag> "<pytest files>" <workload> [<workload> ...]
# A workload is a bench.py argument string in quotes, "" for config 4, e.g.
#   bash exp/ab_round.sh pad "tests/test_gpu_parity.py tests/test_gpu_cfg5.py" "" "--config cfg5"
# (round 5's one-off recipes ab_*.sh are in the history at b6ab0ae)
set -e
T=$1; TESTS=$2; shift 2
O=gpurun_out/ab_$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
i=0
for W in "$@"; do
  timeout -k 10 600 python exp/ab.py --out $O/w$i --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- $W > $O/ab_w$i.txt 2>&1
  i=$((i + 1))
done
tail -n 3 $O/gpu_tests.log; tail -n 2 $O/ab_w*.txt
