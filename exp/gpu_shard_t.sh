set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 && bash exp/gpu_shard_prof2.sh
