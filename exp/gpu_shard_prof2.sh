set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for w in 1 8; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_shard$w -o run -- python3 $GRAFT_REPO_ROOT/exp/shard_prof.py $w > $GRAFT_REPO_ROOT/gpurun_out/prof_shard$w.log 2>&1 || exit 1
done
