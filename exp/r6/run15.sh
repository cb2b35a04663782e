#!/bin/bash
# block zero skip in the 32-bit lane kernel (R_pad 32; lib_w32z.so built with
# GS_W32_ZSKIP=1): the whole -m gpu suite with the variant, then the A/B at
# 2^24 x 32 (the rumor-slice rank's shape at config 4's N = 8)
# (the knob became the default after this run)
set -e
O=gpurun_out/r6_run15; mkdir -p $O
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/safe_gossip_amd/lib_w32z.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
timeout -k 10 600 python exp/ab.py --out $O/ab32 --reps 3 --variant "head:dir=." --variant "w32z:lib=safe_gossip_amd/lib_w32z.so" -- --rumors 32 > $O/ab32.log 2>&1
tail -n 2 $O/ab32.log
