set -o pipefail
mkdir -p gpurun_out
B="--config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cfg5.py -k "delivery_records or faults or config2 or small_gather or cfg5 or many_bins" > gpurun_out/gpu_dlv_w.log 2>&1 &&
timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_cfg5_w.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && ROOT=$GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_cfg5_w -o run -- python3 $ROOT/bench.py $B > $ROOT/gpurun_out/prof_cfg5_w.log 2>&1
