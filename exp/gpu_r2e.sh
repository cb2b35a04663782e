set -o pipefail
mkdir -p gpurun_out/r2e
O=$(pwd)/gpurun_out/r2e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_cfg5.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $O/bench_cfg5.json 2>&1 &&
SAFE_GOSSIP_AMD_NO_DLV=1 timeout -k 10 300 python3 -u bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $O/bench_cfg5_nodlv.json 2>&1 &&
timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-spread > $O/bench_cfg2.json 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg5_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $O/cfg5_trace.log 2>&1
