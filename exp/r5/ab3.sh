#!/bin/bash
# A/B of the DLV partition entry sizes: base tree (12/12 B), head (8/8), head with GS_DLV_FINE12 (8/12)
set -e
O=gpurun_out/r5ab3_${1:-a}; mkdir -p $O
timeout -k 10 600 python exp/ab.py --out $O/cfg5 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." --variant "fine12:lib=exp/lib_fine12.so" -- --config cfg5 > $O/ab_cfg5.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg2 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." --variant "fine12:lib=exp/lib_fine12.so" -- --config cfg2 > $O/ab_cfg2.txt 2>&1
tail -n 3 $O/ab_cfg5.txt
