set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_seq -o run -- python3 bench.py --schedule SEQ --steps 10 --warmup 2 --no-cpu-baseline --no-spread > gpurun_out/prof_seq.log 2>&1
