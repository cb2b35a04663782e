set -o pipefail
mkdir -p gpurun_out/r2t
timeout -k 10 400 python -u -m pytest tests/test_gpu_sliced.py -q --timeout 240 --timeout-method thread > gpurun_out/r2t/gpu_tests_sliced.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-spread > gpurun_out/r2t/bench_default_$i.json 2> gpurun_out/r2t/err || exit 1
timeout -k 10 300 python -u bench.py --sharded --mode slices --no-cpu-baseline --no-spread > gpurun_out/r2t/bench_slices_x1_rccl_$i.json 2>> gpurun_out/r2t/err || exit 1
timeout -k 10 300 python -u bench.py --rumors 32 --no-cpu-baseline --no-spread > gpurun_out/r2t/bench_R32_$i.json 2>> gpurun_out/r2t/err || exit 1
timeout -k 10 300 python -u bench.py --rumors 32 --sharded --mode slices --no-cpu-baseline --no-spread > gpurun_out/r2t/bench_R32_slices_x1_rccl_$i.json 2>> gpurun_out/r2t/err || exit 1
done
