set -o pipefail
# rumor slices on the delivery-record (DLV) kernels: slice parity, then config 5 on one RCCL rank vs unsliced
mkdir -p gpurun_out/slices_dlv
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/slices_dlv/gpu_tests.log 2>&1 || exit 1
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > gpurun_out/slices_dlv/cfg5_plain_$rep.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --config cfg5 --sharded --mode slices --no-cpu-baseline --no-spread > gpurun_out/slices_dlv/cfg5_slices_x1_$rep.json 2>/dev/null || exit 1
done
timeout -k 10 300 python -u bench.py --config cfg5 --rumors 8 --no-cpu-baseline --no-spread > gpurun_out/slices_dlv/cfg5_R8.json 2>/dev/null || exit 1
