set -o pipefail
mkdir -p gpurun_out/r2z
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2z/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2z/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r2z/bench_default.json 2> gpurun_out/r2z/bench_default.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg3 > gpurun_out/r2z/bench_cfg3.json 2> gpurun_out/r2z/bench_cfg3.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg2 > gpurun_out/r2z/bench_cfg2.json 2> gpurun_out/r2z/bench_cfg2.err || exit 1
