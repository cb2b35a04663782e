#!/bin/bash
# round kernel at 5 waves per SIMD (spilling) / without the tail prefetches, config 4
set -e
O=gpurun_out/r6_run10; mkdir -p $O
timeout -k 10 800 python exp/ab.py --out $O/ab --reps 3 --variant "head:dir=." --variant "w5:lib=safe_gossip_amd/lib_w5.so" --variant "nopre:lib=safe_gossip_amd/lib_nopre.so" --variant "w5pre:lib=safe_gossip_amd/lib_w5pre.so" > $O/ab.log 2>&1
tail -n 4 $O/ab.log
