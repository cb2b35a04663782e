set -o pipefail
mkdir -p gpurun_out
GS_BENCH_SHARE_GPU=1 NCCL_DEBUG=WARN timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-spread --nodes 4194304 > gpurun_out/bench2_rccl_shared.log 2>&1
echo "exit $?" >> gpurun_out/bench2_rccl_shared.log
