set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_seq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --schedule SEQ --steps 10 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/gpurun_out/prof_seq.log 2>&1
