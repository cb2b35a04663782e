set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg5.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1 || exit 1
B="--steps 20 --warmup 3 --no-cpu-baseline --no-spread"
out=gpurun_out/ab_filter3.log
: > $out
run() {  # tag lib filter
  echo "$1" >> $out
  SAFE_GOSSIP_AMD_LIB=$PWD/exp/lib_$2.so SAFE_GOSSIP_AMD_FILTER=$3 timeout -k 10 200 python -u bench.py $B >> $out 2>&1
}
for i in 1 2; do
  run "prod f0" prod 0 || exit 1
  run "prod f1" prod 1 || exit 1
  run "branch" fbr 1 || exit 1
  run "noacct" fnoacct 1 || exit 1
  run "branch+noacct" fbrnoacct 1 || exit 1
done
echo "cfg5 prod" >> $out
SAFE_GOSSIP_AMD_LIB=$PWD/exp/lib_prod.so timeout -k 10 300 python -u bench.py --config cfg5 $B >> $out 2>&1
