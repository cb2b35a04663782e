set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r2r gpurun_out/prof_r2r_cfg5
timeout -k 10 400 python -u -m pytest tests/test_gpu_sliced.py -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_sliced.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
for R in 128 64 32; do
timeout -k 10 200 python -u bench.py --rumors $R --no-cpu-baseline --no-spread > gpurun_out/bench_cfg4_R$R.json 2> gpurun_out/bench_cfg4_R$R.err || exit 1
done
timeout -k 10 300 python -u bench.py --sharded --mode slices --no-cpu-baseline > gpurun_out/bench_slices_x1_rccl.json 2> gpurun_out/bench_slices_x1_rccl.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1 --no-cpu-baseline --no-spread > gpurun_out/bench2_gloo_slices.json 2> gpurun_out/bench2_gloo_slices.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg3 > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg2 > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r2r > gpurun_out/prof_r2r.log 2>&1 || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r2r_cfg5 --config cfg5 > gpurun_out/prof_r2r_cfg5.log 2>&1 || exit 1
