set -o pipefail
# in-list sort blocks per bin for small networks (config 3: 2^20 nodes = 64 bins):
# adaptive (4 per bin below 128 bins) vs one per bin; parity suite first with the adaptive library
mkdir -p gpurun_out/ab_small3
L=safe_gossip_amd/libsafe_gossip_amd.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ab_small3/gpu_tests.log 2>&1 || exit 1
cp $L exp/ab/head.so
for rep in 1 2 3; do
for v in chunkfixed adaptive; do
  cp exp/ab/$v.so $L
  timeout -k 10 120 python -u bench.py --config cfg3 --no-cpu-baseline --no-spread > gpurun_out/ab_small3/cfg3_${v}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --no-spread > gpurun_out/ab_small3/cfg2_${v}_$rep.json 2>/dev/null || exit 1
done
done
cp exp/ab/head.so $L
