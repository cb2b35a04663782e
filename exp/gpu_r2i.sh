set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sparse" > gpurun_out/gpu_sparse.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/gpu_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_sparse.log 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=dense timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_dense.log 2>&1
