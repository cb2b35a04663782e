set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg5.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1 || exit 1
B="--steps 20 --warmup 3 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_filter6.log
: > $out
for i in 1 2; do
  for f in 1 0; do
    echo "filter=$f run $i" >> $out
    SAFE_GOSSIP_AMD_FILTER=$f timeout -k 10 200 python -u bench.py $B >> $out 2>&1 || exit 1
  done
done
rm -rf gpurun_out/prof_r3 gpurun_out/prof_r3_cfg5
timeout -k 10 700 bash profiles/rocprof_r2.sh r3 > gpurun_out/prof_r3.log 2>&1 || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r3_cfg5 --config cfg5 > gpurun_out/prof_r3_cfg5.log 2>&1 || exit 1
