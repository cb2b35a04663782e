#!/bin/bash
# the rumor-slice shapes of config 4 on one GPU (2^24 x 256/N): in-list build in sequence (default) vs beside the round kernel
set -e
O=gpurun_out/r4sconc; mkdir -p $O
for i in 1 2; do
  for R in 32 64 128; do
    timeout -k 10 200 python bench.py --rumors $R --no-cpu-baseline --no-spread > $O/r${R}_seq_$i.json 2>>$O/err.log
    SAFE_GOSSIP_AMD_CONCURRENT_INLISTS=1 timeout -k 10 200 python bench.py --rumors $R --no-cpu-baseline --no-spread > $O/r${R}_conc_$i.json 2>>$O/err.log
  done
done
