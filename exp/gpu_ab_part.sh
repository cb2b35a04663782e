set -o pipefail
# A/B of the DLV build's partition chunk (sources per dl_coarse / dl_fine block) at config 5
mkdir -p gpurun_out/ab_part
L=safe_gossip_amd/libsafe_gossip_amd.so
cp $L exp/ab/head.so
for rep in 1 2 3; do
for v in ${VARIANTS:-base part4k}; do
  cp exp/ab/$v.so $L
  timeout -k 10 200 python -u bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu-baseline --no-spread > gpurun_out/ab_part/${v}_$rep.json 2>/dev/null || exit 1
done
done
cp exp/ab/head.so $L
