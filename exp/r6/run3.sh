#!/bin/bash
# 64- vs 128-lane round-kernel blocks (config 4, config 3); config 3 against the round-5 tree
set -e
O=gpurun_out/r6_run3; mkdir -p $O
timeout -k 10 600 python exp/ab.py --out $O/ab64 --reps 3 --variant "b128:dir=." --variant "b64:lib=safe_gossip_amd/lib_blk64.so" > $O/ab64.log 2>&1
tail -n 2 $O/ab64.log
timeout -k 10 400 python exp/ab.py --out $O/ab64_cfg3 --reps 3 --variant "base:dir=exp/base_tree" --variant "b128:dir=." --variant "b64:lib=safe_gossip_amd/lib_blk64.so" -- --config cfg3 > $O/ab64_cfg3.log 2>&1
tail -n 3 $O/ab64_cfg3.log
