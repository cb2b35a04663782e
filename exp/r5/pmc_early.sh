#!/bin/bash
# SQ counters of config 4's round kernel over the first 6 rounds only (the latency-bound early rounds)
set -e
O=gpurun_out/pmc_early_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-spread --pmc off"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- $B > $O/tr.log 2>&1
ls $O
