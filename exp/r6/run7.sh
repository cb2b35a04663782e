#!/bin/bash
# 32-bit lane kernel (R_pad 32: the 8-GPU slice shape of config 4): 256- vs 128- vs 64-lane blocks
set -e
O=gpurun_out/r6_run7; mkdir -p $O
timeout -k 10 600 python exp/ab.py --out $O/ab_r32 --reps 3 --variant "w256:dir=." --variant "w128:lib=safe_gossip_amd/lib_w128.so" --variant "w64:lib=safe_gossip_amd/lib_w64.so" -- --rumors 32 > $O/ab_r32.log 2>&1
tail -n 3 $O/ab_r32.log
