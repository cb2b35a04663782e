#!/bin/bash
# zero-wave load skip (per-wave all-A words): parity with the variant library, then the A/B (config 4, config 3)
# (the variant -- GS_RK_ZLOAD=1: a per-wave all-A word written by each launch and
#  read with a scalar load before the stage loads -- was measured slower and its code removed;
#  results in profiles/r6/rejected_zload/)
set -e
O=gpurun_out/r6_run13; mkdir -p $O
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/safe_gossip_amd/lib_zload.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense_check.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not config5 and not multi_gpu_shapes" > $O/tests.log 2>&1
tail -n 2 $O/tests.log
timeout -k 10 600 python exp/ab.py --out $O/ab --reps 3 --variant "head:dir=." --variant "zload:lib=safe_gossip_amd/lib_zload.so" > $O/ab.log 2>&1
tail -n 2 $O/ab.log
timeout -k 10 300 python exp/ab.py --out $O/ab3 --reps 3 --variant "head:dir=." --variant "zload:lib=safe_gossip_amd/lib_zload.so" -- --config cfg3 > $O/ab3.log 2>&1
tail -n 2 $O/ab3.log
