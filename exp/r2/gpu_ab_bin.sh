set -o pipefail
# A/B of library variants: exp/ab/<variant>.so are built beforehand on the CPU host
# (build.py's hipcc line plus the variant's -D switch) and swapped in per run.
mkdir -p gpurun_out
L=safe_gossip_amd/libsafe_gossip_amd.so
for rep in 1 2 3; do
for v in base bin13 bin15; do
  cp exp/ab/$v.so $L
  echo "== $v" >> gpurun_out/ab_bin.log
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spread >> gpurun_out/ab_bin.log 2>&1 || exit 1
done
done
