#!/bin/bash
# three-way interleaved timing: exp/base_tree, this tree, exp/var_tree (no parity run)
#   bash exp/ab3.sh <tag> <workload> [<workload> ...]
set -e
T=$1; shift
O=gpurun_out/ab3_$T; mkdir -p $O
i=0
for W in "$@"; do
  timeout -k 10 600 python exp/ab.py --out $O/w$i --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." --variant "var:dir=exp/var_tree" -- $W > $O/ab_w$i.txt 2>&1
  i=$((i + 1))
done
tail -n 3 $O/ab_w*.txt
