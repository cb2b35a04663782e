#!/bin/bash
# DLV-path tests, then A/B (base tree vs HEAD) at configs 2 and 5
set -e
O=gpurun_out/r5dlv_${1:-a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "delivery or dlv or cfg5 or config5 or config2 or digest_small or sliced or packed or long_run or small_gather" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg2 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg2 > $O/ab_cfg2.txt 2>&1
timeout -k 10 400 python exp/ab.py --out $O/cfg5 --reps 2 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg5 > $O/ab_cfg5.txt 2>&1
tail -n 2 $O/tests.log
