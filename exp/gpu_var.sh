set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
SAFE_GOSSIP_AMD_GENERIC_INLISTS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_generic.log 2>&1 &&
bash exp/run_variants.sh prod prod > gpurun_out/variants.txt 2>&1 &&
bash exp/gpu_prof.sh prod
