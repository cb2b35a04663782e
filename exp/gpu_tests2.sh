set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 ./examples/one_message_test 2000 200 > gpurun_out/one_message_2000_seq.log 2>&1 &&
timeout -k 10 200 ./examples/one_message_test 20 1000 > gpurun_out/one_message_20_seq.log 2>&1
