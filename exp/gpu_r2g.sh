set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wire.py tests/test_gpu_facade.py > gpurun_out/gpu_wire.log 2>&1
