#!/bin/bash
# Round 3: localise the single-part stall (gloo vs RCCL, serialised kernels,
# two parts as control), then the pipe A/B.
set -o pipefail
OUT=gpurun_out/r3_batch4
mkdir -p $OUT
timeout -k 10 150 python -u exp/r3/rccl_p1.py 24 1 256 gloo > $OUT/p1_gloo.log 2>&1; echo "p1 gloo rc=$?"; grep -v WARN $OUT/p1_gloo.log | tail -3
timeout -k 10 150 python -u exp/r3/rccl_p1.py 24 2 256 nccl > $OUT/p2_nccl.log 2>&1; echo "p2 nccl rc=$?"; grep -v WARN $OUT/p2_nccl.log | tail -3
AMD_SERIALIZE_KERNEL=3 timeout -k 10 150 python -u exp/r3/rccl_p1.py 24 1 256 nccl > $OUT/p1_nccl_serial.log 2>&1; echo "p1 nccl serialized rc=$?"; grep -v WARN $OUT/p1_nccl_serial.log | tail -3
AMD_LOG_LEVEL=3 timeout -k 10 150 python -u exp/r3/rccl_p1.py 24 1 256 nccl > $OUT/p1_nccl_log3.log 2>&1; echo "p1 nccl log3 rc=$?"; grep -v WARN $OUT/p1_nccl_log3.log | grep -v "^$" | tail -3
gzip -f $OUT/p1_nccl_log3.log
bash exp/r3/ab_pipe2.sh
