#!/bin/bash
# Quiet-wave fast path + zero-node maps: parity, then A/B of config 4 (base tree, HEAD, HEAD without maps) and config 3
set -e
T=${1:-a}
O=gpurun_out/r5q_$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense_check.py tests/test_gpu_wire.py tests/test_gpu_api.py tests/test_gpu_harness.py tests/test_gpu_sliced.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 600 python exp/ab.py --out $O/cfg4 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." --variant "nozmap:env=SAFE_GOSSIP_AMD_ZMAP=0" -- > $O/ab_cfg4.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg3 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg3 > $O/ab_cfg3.txt 2>&1
tail -n 3 $O/gpu_tests.log; tail -n 3 $O/ab_cfg4.txt $O/ab_cfg3.txt
