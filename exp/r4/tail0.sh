#!/bin/bash
# config 4 gather round kernel: the first tail pusher id read with the batch (tail0) vs head; parity of the tail0 build, then interleaved A/B at config 4
set -e
O=gpurun_out/r4tail0; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_tail0.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_parity.py > $O/tests_tail0.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_head_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_tail0.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_tail0_$i.json 2>>$O/err.log
done
