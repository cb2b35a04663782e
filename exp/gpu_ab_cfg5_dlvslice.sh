set -o pipefail
# config 5 before / after the slice counts in gs_dlv4 (interleaved, one box)
mkdir -p gpurun_out/ab_cfg5_dlvslice
L=safe_gossip_amd/libsafe_gossip_amd.so
cp $L exp/ab/head.so
for rep in 1 2 3; do
for v in predlvslice head_dlvslice; do
  cp exp/ab/$v.so $L
  timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > gpurun_out/ab_cfg5_dlvslice/${v}_$rep.json 2>/dev/null || exit 1
done
done
cp exp/ab/head.so $L
