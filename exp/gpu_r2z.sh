set -o pipefail
mkdir -p gpurun_out
B="--config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_dlv4_z.log
: > $out
SAFE_GOSSIP_AMD_DLV_PACK=u32x1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "delivery_records_packed or faults" > gpurun_out/gpu_dlv_z.log 2>&1 &&
for i in 1 2; do
echo "u32x2 $i" >> $out; timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
echo "u32x1 $i" >> $out; SAFE_GOSSIP_AMD_DLV_PACK=u32x1 timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
done
