#!/bin/bash
# Timing-only variants of inl_sort_dlv at config 5 (results wrong, memory-safe): what the per-target insertion sort and the pull loop cost
set -e
O=gpurun_out/r5sp_${1:-a}; mkdir -p $O
timeout -k 10 600 python exp/ab.py --out $O/cfg5 --reps 2 --variant "head:dir=." --variant "noisort:lib=exp/r5/libs/exp_GS_EXP_NOISORT.so" --variant "nopull:lib=exp/r5/libs/exp_GS_EXP_NOPULL.so" -- --config cfg5 > $O/ab_cfg5.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in NOISORT NOPULL; do
  SAFE_GOSSIP_AMD_LIB=exp/r5/libs/exp_GS_EXP_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-spread --pmc off > $O/prof_$v.log 2>&1
done
tail -n 4 $O/ab_cfg5.txt
