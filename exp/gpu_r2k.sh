set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/pmc_valu
cd /tmp && export TMPDIR=/tmp
export SAFE_GOSSIP_AMD_LIB=$ROOT/exp/lib_head.so
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $ROOT/gpurun_out/pmc_valu/head -o run -- python3 $ROOT/exp/ab_sparse.py 16777216 256 8 head > $ROOT/gpurun_out/pmc_valu/head.log 2>&1
unset SAFE_GOSSIP_AMD_LIB
export SAFE_GOSSIP_AMD_SPARSE=on
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $ROOT/gpurun_out/pmc_valu/on -o run -- python3 $ROOT/exp/ab_sparse.py 16777216 256 8 new > $ROOT/gpurun_out/pmc_valu/on.log 2>&1
