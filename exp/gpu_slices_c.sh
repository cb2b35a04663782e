set -o pipefail
mkdir -p gpurun_out/r2s
timeout -k 10 400 python -u -m pytest tests/test_gpu_sliced.py -v --timeout 240 --timeout-method thread > gpurun_out/r2s/gpu_tests_sliced.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --sharded --mode slices --no-cpu-baseline --no-spread > gpurun_out/r2s/bench_slices_x1_rccl.json 2> gpurun_out/r2s/bench_slices_x1_rccl.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-spread > gpurun_out/r2s/bench_default.json 2> gpurun_out/r2s/bench_default.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r2s/bench2_gloo_slices.json 2> gpurun_out/r2s/bench2_gloo_slices.err || exit 1
