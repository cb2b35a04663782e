set -o pipefail
# per-kernel times of library variants (timing only): rocprofv3 kernel trace of the bench window
mkdir -p gpurun_out/ab_prof
L=safe_gossip_amd/libsafe_gossip_amd.so
cp $L exp/ab/head.so
ROOT=$(pwd)
for v in ${VARIANTS:-base nosib}; do
  cp exp/ab/$v.so $L
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/ab_prof/$v -o run -- python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spread $BENCH_ARGS > $ROOT/gpurun_out/ab_prof/$v.log 2>&1) || exit 1
done
cp exp/ab/head.so $L
