set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u exp/shard_diag.py gloo 1 256 16 20 22 24 > gpurun_out/diag_gloo.log 2>&1
timeout -k 10 120 python -u exp/shard_diag.py nccl 1 256 16 20 22 24 > gpurun_out/diag_nccl1.log 2>&1
timeout -k 10 120 python -u exp/shard_diag.py nccl 2 256 16 20 22 24 > gpurun_out/diag_nccl2.log 2>&1
exit 0
