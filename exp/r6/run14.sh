#!/bin/bash
# block-level zero skip (256-lane gather transitions GS_RK_ZSKIP_BLK=1, packed
# DLV kernel GS_DLV4_ZSKIP=1; lib_zblk.so built with both): the whole -m gpu
# suite with the variant library, then the A/B on configs 5, 2 and 4
# (both knobs became the defaults after this run)
set -e
O=gpurun_out/r6_run14; mkdir -p $O
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/safe_gossip_amd/lib_zblk.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
timeout -k 10 600 python exp/ab.py --out $O/ab5 --reps 3 --variant "head:dir=." --variant "zblk:lib=safe_gossip_amd/lib_zblk.so" -- --config cfg5 > $O/ab5.log 2>&1
tail -n 2 $O/ab5.log
timeout -k 10 300 python exp/ab.py --out $O/ab2 --reps 3 --variant "head:dir=." --variant "zblk:lib=safe_gossip_amd/lib_zblk.so" -- --config cfg2 > $O/ab2.log 2>&1
tail -n 2 $O/ab2.log
