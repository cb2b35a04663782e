set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/pmc_valu2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wire.py > gpurun_out/gpu_parity_l.log 2>&1 || exit 1
out=gpurun_out/ab_sparse2.log
: > $out
SAFE_GOSSIP_AMD_LIB=exp/lib_head.so timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 head >> $out 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=dense timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 new >> $out 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=auto timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 new >> $out 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=on timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 new >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for m in dense on; do
SAFE_GOSSIP_AMD_SPARSE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $ROOT/gpurun_out/pmc_valu2/$m -o run -- python3 $ROOT/exp/ab_sparse.py 16777216 256 8 new > $ROOT/gpurun_out/pmc_valu2/$m.log 2>&1 || exit 1
done
