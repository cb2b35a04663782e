set -o pipefail
# AMDGPU machine-scheduler strategies for the whole library (timing A/B, interleaved, one box)
mkdir -p gpurun_out/ab_sched
L=safe_gossip_amd/libsafe_gossip_amd.so
cp $L exp/ab/head.so
for rep in 1 2 3; do
for v in base ilp memclause; do
  cp exp/ab/$v.so $L
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-spread > gpurun_out/ab_sched/cfg4_${v}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python -u bench.py --rumors 32 --no-cpu-baseline --no-spread > gpurun_out/ab_sched/R32_${v}_$rep.json 2>/dev/null || exit 1
done
done
cp exp/ab/head.so $L
