#!/bin/bash
# packed DLV kernel: 256- vs 128- vs 64-lane blocks (config 5, config 2)
set -e
O=gpurun_out/r6_run6; mkdir -p $O
timeout -k 10 600 python exp/ab.py --out $O/ab_cfg5 --reps 3 --variant "d256:dir=." --variant "d128:lib=safe_gossip_amd/lib_dlv128.so" --variant "d64:lib=safe_gossip_amd/lib_dlv64.so" -- --config cfg5 > $O/ab_cfg5.log 2>&1
tail -n 3 $O/ab_cfg5.log
timeout -k 10 300 python exp/ab.py --out $O/ab_cfg2 --reps 3 --variant "d256:dir=." --variant "d128:lib=safe_gossip_amd/lib_dlv128.so" --variant "d64:lib=safe_gossip_amd/lib_dlv64.so" -- --config cfg2 > $O/ab_cfg2.log 2>&1
tail -n 3 $O/ab_cfg2.log
