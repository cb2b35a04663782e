#!/bin/bash
# Round 3: is the single-part stall an RCCL size threshold (2^30 bytes)?
set -o pipefail
OUT=gpurun_out/r3_batch5
mkdir -p $OUT
timeout -k 10 150 python -u exp/r3/rccl_size.py 256 512 1000 1024 1025 1100 1200 > $OUT/rccl_size.log 2>&1; echo "rccl_size rc=$?"; grep -v "WARN\|^$" $OUT/rccl_size.log | tail -16
timeout -k 10 120 python -u exp/r3/rccl_p1.py 23 1 256 nccl > $OUT/p1_n23.log 2>&1; echo "p1 2^23 rc=$?"; grep -v "WARN\|^$" $OUT/p1_n23.log | tail -3
