set -o pipefail
mkdir -p gpurun_out
B="--config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_split_aa.log
: > $out
SAFE_GOSSIP_AMD_LIB=exp/lib_split2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "delivery_records or faults" > gpurun_out/gpu_split_aa.log 2>&1 &&
SAFE_GOSSIP_AMD_LIB=exp/lib_split3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "delivery_records or faults" >> gpurun_out/gpu_split_aa.log 2>&1 &&
for i in 1 2; do
for v in split2 split3; do
echo "$v $i" >> $out; SAFE_GOSSIP_AMD_LIB=exp/lib_$v.so timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
done
echo "head $i" >> $out; timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
done
