#!/bin/bash
# issue priority by phase in the 32-bit lane kernel (R_pad 32): parity, then A/B of 2^24 x 32 and 2^20 x 32
set -e
O=gpurun_out/ab_w32p; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sliced.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 500 python exp/ab.py --out $O/s32 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --rumors 32 > $O/ab_s32.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/m32 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --nodes 1048576 --rumors 32 > $O/ab_m32.txt 2>&1
tail -n 3 $O/gpu_tests.log; tail -n 2 $O/ab_s32.txt $O/ab_m32.txt
