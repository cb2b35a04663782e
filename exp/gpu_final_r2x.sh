set -o pipefail
mkdir -p gpurun_out/r2x
rm -rf gpurun_out/prof_r2x gpurun_out/prof_r2x_cfg5
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2x/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2x/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r2x/bench_default.json 2> gpurun_out/r2x/bench_default.err || exit 1
timeout -k 10 400 python -u bench.py --config cfg5 > gpurun_out/r2x/bench_cfg5.json 2> gpurun_out/r2x/bench_cfg5.err || exit 1
for R in 128 64 32; do
timeout -k 10 200 python -u bench.py --rumors $R --no-cpu-baseline --no-spread > gpurun_out/r2x/bench_cfg4_R$R.json 2> gpurun_out/r2x/bench_cfg4_R$R.err || exit 1
done
timeout -k 10 300 python -u bench.py --sharded --mode slices --no-cpu-baseline > gpurun_out/r2x/bench_slices_x1_rccl.json 2> gpurun_out/r2x/bench_slices_x1_rccl.err || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r2x > gpurun_out/prof_r2x.log 2>&1 || exit 1
timeout -k 10 700 bash profiles/rocprof_r2.sh r2x_cfg5 --config cfg5 > gpurun_out/prof_r2x_cfg5.log 2>&1 || exit 1
