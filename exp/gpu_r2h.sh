set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u exp/round_profile.py > gpurun_out/round_profile.log 2>&1
