set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/gpu_all_n.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_n.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cfg5_n.log 2>&1 &&
bash profiles/rocprof_r2.sh r2n &&
bash profiles/rocprof_r2.sh r2n_cfg5 --config cfg5
