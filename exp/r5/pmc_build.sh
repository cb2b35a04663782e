#!/bin/bash
# SQ counters of config 5's build kernels (two passes), for where inl_sort_dlv / dl_* spend their cycles
set -e
O=gpurun_out/pmc_build_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --config cfg5 --steps 3 --warmup 2 --no-cpu-baseline --no-spread --pmc off"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1
ls -R $O | head -20
