set -o pipefail
mkdir -p gpurun_out/dlv_check
timeout -k 10 600 python -u -m pytest tests -m gpu -k "delivery or cfg5 or config5 or fullsize or full_size or dlv or small" -v --timeout 300 --timeout-method thread > gpurun_out/dlv_check/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config cfg5 > gpurun_out/dlv_check/bench_cfg5.json 2> gpurun_out/dlv_check/bench_cfg5.err || exit 1
