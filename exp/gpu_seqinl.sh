set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spread > gpurun_out/bench_quick.log 2>&1 &&
timeout -k 10 200 python -u bench.py --schedule SEQ --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_seq.log 2>&1
