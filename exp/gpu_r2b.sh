set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_shard.log 2>&1 &&
timeout -k 10 300 python -u exp/shard_prof.py 8 > gpurun_out/shard_prof8.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/shardprof8 -o run -- python3 -u exp/shard_prof.py 8 > gpurun_out/shard_prof8_rocprof.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-spread --dist-backend gloo --nodes 4194304 > gpurun_out/bench2_gloo.log 2>&1
