#!/bin/bash
# config 4 gather round kernel: the second tail pusher id read with the batch too (tail1) vs HEAD; parity of tail1, then interleaved A/B at config 4
set -e
O=gpurun_out/r4tail1; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_tail1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_parity.py > $O/tests_tail1.log 2>&1
for i in 1 2 3; do
  for v in base tail1; do
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_${v}_$i.json 2>>$O/err.log
  done
done
