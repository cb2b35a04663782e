set -o pipefail
mkdir -p gpurun_out
B="--config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_dlv4_v.log
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "delivery_records or faults or config2 or small_gather or harness" > gpurun_out/gpu_dlv4_v.log 2>&1 &&
for i in 1 2; do
echo "head $i" >> $out; timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
echo "w4 $i" >> $out; SAFE_GOSSIP_AMD_LIB=exp/lib_dlv4_w4.so timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
done
echo "cfg2" >> $out; timeout -k 10 200 python -u bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-spread >> $out 2>&1
