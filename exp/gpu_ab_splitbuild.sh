set -o pipefail
# Two-phase in-list build (SAFE_GOSSIP_AMD_SPLIT_BUILD=1: inl_bin beside the round kernel on the side
# stream) vs in sequence: parity with it on, then interleaved benches (config 4 and R = 32)
mkdir -p gpurun_out/ab_splitbuild
SAFE_GOSSIP_AMD_SPLIT_BUILD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_api.py tests/test_gpu_sliced.py -q -x --timeout 240 --timeout-method thread > gpurun_out/ab_splitbuild/parity_on.log 2>&1 || exit 1
for rep in 1 2 3; do
for v in 0 1; do
  SAFE_GOSSIP_AMD_SPLIT_BUILD=$v timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-spread > gpurun_out/ab_splitbuild/cfg4_sb${v}_$rep.json 2>/dev/null || exit 1
  SAFE_GOSSIP_AMD_SPLIT_BUILD=$v timeout -k 10 120 python -u bench.py --rumors 32 --no-cpu-baseline --no-spread > gpurun_out/ab_splitbuild/R32_sb${v}_$rep.json 2>/dev/null || exit 1
done
done
