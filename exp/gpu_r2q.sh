set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 200 python -u bench.py --sharded --parts 2 --no-cpu-baseline --no-spread > gpurun_out/bench_sh2_q.log 2>&1 &&
timeout -k 10 200 python -u bench.py --sharded --parts 4 --no-cpu-baseline --no-spread > gpurun_out/bench_sh4_q.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/prof_sh2 -o run -- python3 $ROOT/bench.py --sharded --parts 2 --steps 6 --warmup 1 --no-cpu-baseline --no-spread > $ROOT/gpurun_out/prof_sh2.log 2>&1
