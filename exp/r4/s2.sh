#!/bin/bash
# config 4 gather round kernel: the row of sibling #kBatchE issued right after the batch (s2) vs t0row (the first tail pusher row prefetch); parity of s2, then interleaved A/B at config 4
set -e
O=gpurun_out/r4s2; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_s2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_parity.py > $O/tests_s2.log 2>&1
for i in 1 2 3; do
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_t0row.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_t0row_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_s2.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_s2_$i.json 2>>$O/err.log
done
