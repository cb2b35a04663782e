set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_shard -o run -- python3 $GRAFT_REPO_ROOT/exp/shard_prof.py 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_shard.log 2>&1
