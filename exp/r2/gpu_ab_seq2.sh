set -o pipefail
# A/B of library variants: exp/ab/<variant>.so are built beforehand on the CPU host
# (build.py's hipcc line plus the variant's -D switch) and swapped in per run.
mkdir -p gpurun_out
L=safe_gossip_amd/libsafe_gossip_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -x -q -k "seq or one_message or generic" --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
for v in new head; do
  cp exp/ab/$v.so $L
  echo "== $v" >> gpurun_out/ab_seq2.log
  timeout -k 10 120 python -u bench.py --schedule SEQ --steps 20 --warmup 3 --no-cpu-baseline --no-spread >> gpurun_out/ab_seq2.log 2>&1 || exit 1
done
done
