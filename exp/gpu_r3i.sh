set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r3 > gpurun_out/prof_r3.log 2>&1 || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r3_cfg5 --config cfg5 > gpurun_out/prof_r3_cfg5.log 2>&1 || exit 1
