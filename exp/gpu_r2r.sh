set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py > gpurun_out/gpu_shard_r.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1 --no-spread --nodes 4194304 > gpurun_out/bench_gloo2_r.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --parts 2 --steps 5 --warmup 1 --nodes 4194304 > gpurun_out/bench_gloo2p2_r.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $ROOT/gpurun_out/pmc_cfg5 -o run -- python3 $ROOT/bench.py --config cfg5 --steps 4 --warmup 1 --no-cpu-baseline --no-spread > $ROOT/gpurun_out/pmc_cfg5.log 2>&1
