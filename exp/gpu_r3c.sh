set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
B="--steps 20 --warmup 3 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_filter.log
: > $out
for i in 1 2; do
  for f in 1 0; do
    echo "filter=$f run $i" >> $out
    SAFE_GOSSIP_AMD_FILTER=$f timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
  done
done
