set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in sprod sseq; do
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/exp/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sv_$v -o run -- python3 $GRAFT_REPO_ROOT/exp/shard_prof.py 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_sv_$v.log 2>&1 || exit 1
done
