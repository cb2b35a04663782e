set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/pmc_filt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg5.py tests/test_gpu_wire.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1 || exit 1
B="--steps 20 --warmup 3 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_filter4.log
: > $out
for i in 1 2; do
  for f in 1 0; do
    echo "filter=$f run $i" >> $out
    SAFE_GOSSIP_AMD_FILTER=$f timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
SAFE_GOSSIP_AMD_FILTER=$f timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $ROOT/gpurun_out/pmc_filt/f$f -o run -- python3 $ROOT/bench.py --steps 16 --warmup 0 --no-cpu-baseline --no-spread > $ROOT/gpurun_out/pmc_filt/f$f.log 2>&1 || exit 1
done
