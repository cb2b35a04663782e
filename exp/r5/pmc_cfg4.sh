#!/bin/bash
# SQ counters of config 4's round kernel and builds (two passes)
set -e
O=gpurun_out/pmc_cfg4_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-spread --pmc off"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SMEM -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1
ls $O
