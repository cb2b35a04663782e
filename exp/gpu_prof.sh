set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/exp/lib_${1}.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/gpurun_out/prof_$1.log 2>&1
