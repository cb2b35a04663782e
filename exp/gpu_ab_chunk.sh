set -o pipefail
# A/B of in-list build chunk sizes: exp/ab/<variant>.so built on the CPU host with
# build.build_engine(defines=[...]) and swapped in per run (interleaved, one box)
mkdir -p gpurun_out/${OUT:-ab_chunk}
L=safe_gossip_amd/libsafe_gossip_amd.so
cp $L exp/ab/head.so
for rep in 1 2 3; do
for v in ${VARIANTS:-base split1}; do
  cp exp/ab/$v.so $L
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spread > gpurun_out/${OUT:-ab_chunk}/${v}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python -u bench.py --rumors 32 --steps 20 --warmup 3 --no-cpu-baseline --no-spread > gpurun_out/${OUT:-ab_chunk}/R32_${v}_$rep.json 2>/dev/null || exit 1
done
done
cp exp/ab/head.so $L
