set -o pipefail
mkdir -p gpurun_out
SAFE_GOSSIP_AMD_CONCURRENT_INLISTS=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spread > gpurun_out/bench_conc.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg5.log 2>&1
