set -o pipefail
mkdir -p gpurun_out
B="--config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_dlv4_y.log
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cfg5.py tests/test_gpu_harness.py -k "delivery_records or faults or config2 or small_gather or cfg5 or many_bins or harness or one_message" > gpurun_out/gpu_dlv_y.log 2>&1 &&
for i in 1 2; do
echo "u32 $i" >> $out; timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
echo "u64 $i" >> $out; SAFE_GOSSIP_AMD_DLV_PACK=u64 timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
done
echo "cfg2 u32" >> $out; timeout -k 10 200 python -u bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-spread >> $out 2>&1
