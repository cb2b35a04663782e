#!/bin/bash
# the DLV round kernel's tail prefetch: two codes (head) vs three codes bound to 7 waves per SIMD vs two codes bound to 7 waves; parity of the three-code build, then interleaved A/B at config 5
set -e
O=gpurun_out/r4pre3; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pre3w7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py -k "config5 or small" > $O/tests_pre3.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_head_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pre3w7.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_pre3w7_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pre2w7.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_pre2w7_$i.json 2>>$O/err.log
done
