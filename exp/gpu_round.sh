# Full validation of the current tree on the GPU box: gpu tests, smoke, the
# default bench line, then the rocprof trace + PMC passes (tag $1).
set -o pipefail
TAG=${1:-r1e}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 &&
bash profiles/rocprof_r1.sh $TAG
