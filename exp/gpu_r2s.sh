set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "delivery_records or faults or config2 or small_gather" > gpurun_out/gpu_dlv4_s.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/gpu_all_s.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cfg5_s.log 2>&1 &&
SAFE_GOSSIP_AMD_DLV_PACK=0 timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread > gpurun_out/bench_cfg5_nopack_s.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cfg2_s.log 2>&1
