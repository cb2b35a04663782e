#!/bin/bash
# DLV parity + shards, then A/B of configs 5 and 2 (base tree vs HEAD): pushers ordered by a comparator network instead of insertion sort (and config 4)
set -e
T=${1:-a}
O=gpurun_out/r5rank_$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg5.py tests/test_gpu_dense_check.py tests/test_gpu_wire.py tests/test_gpu_sharded.py tests/test_gpu_sliced.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python exp/ab.py --out $O/cfg5 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg5 > $O/ab_cfg5.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg2 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg2 > $O/ab_cfg2.txt 2>&1
timeout -k 10 500 python exp/ab.py --out $O/cfg4 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- > $O/ab_cfg4.txt 2>&1
tail -n 3 $O/ab_cfg4.txt; tail -n 3 $O/gpu_tests.log $O/ab_cfg5.txt $O/ab_cfg2.txt
