set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_r3b.log
for i in 1 2 3; do
  bash exp/run_variants.sh early late chunk8k nosib >> gpurun_out/ab_r3b.log 2>&1 || exit 1
done
