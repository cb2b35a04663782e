set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
B="--config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_dlv4_u.log
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "delivery_records or faults or config2 or small_gather" > gpurun_out/gpu_dlv4_u.log 2>&1 &&
for i in 1 2; do
echo "head $i" >> $out; timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
echo "w4 $i" >> $out; SAFE_GOSSIP_AMD_LIB=exp/lib_dlv4_w4.so timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
done
echo "nofaults" >> $out; timeout -k 10 200 python -u bench.py $B --churn 0 --drop-push 0 --drop-pull 0 >> $out 2>&1 || exit 1
echo "nofaults-nopack" >> $out; SAFE_GOSSIP_AMD_DLV_PACK=0 timeout -k 10 200 python -u bench.py $B --churn 0 --drop-push 0 --drop-pull 0 >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $ROOT/gpurun_out/pmc_cfg5p -o run -- python3 $ROOT/bench.py --config cfg5 --steps 4 --warmup 1 --no-cpu-baseline --no-spread > $ROOT/gpurun_out/pmc_cfg5p.log 2>&1
