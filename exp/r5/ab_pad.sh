#!/bin/bash
# Round kernel change: parity, then A/B of configs 4 and 3 (base tree vs HEAD), and SQ LDS counters
set -e
T=${1:-a}
O=gpurun_out/r5pad_$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense_check.py tests/test_gpu_wire.py tests/test_gpu_sharded.py tests/test_gpu_sliced.py tests/test_gpu_cfg5.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 600 python exp/ab.py --out $O/cfg4 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- > $O/ab_cfg4.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg3 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg3 > $O/ab_cfg3.txt 2>&1
timeout -k 10 400 python exp/ab.py --out $O/cfg5 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg5 > $O/ab_cfg5.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg2 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg2 > $O/ab_cfg2.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p1 -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-spread --pmc off > $O/p1.log 2>&1
tail -n 3 $O/gpu_tests.log; tail -n 2 $O/ab_cfg4.txt $O/ab_cfg3.txt $O/ab_cfg5.txt $O/ab_cfg2.txt
