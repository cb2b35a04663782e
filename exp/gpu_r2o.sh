set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py > gpurun_out/gpu_shard_o.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/gpu_all_o.log 2>&1 &&
timeout -k 10 200 python -u bench.py --sharded --parts 1 --no-cpu-baseline --no-spread > gpurun_out/bench_sh1_o.log 2>&1 &&
timeout -k 10 200 python -u bench.py --sharded --parts 2 --no-cpu-baseline --no-spread > gpurun_out/bench_sh2_o.log 2>&1 &&
timeout -k 10 200 python -u bench.py --sharded --parts 4 --no-cpu-baseline --no-spread > gpurun_out/bench_sh4_o.log 2>&1
