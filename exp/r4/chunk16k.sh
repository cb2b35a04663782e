#!/bin/bash
# config 4 in-list build: inl_bin chunks of 16 K sources (one block per CU, half the fill reservations, runs twice as long) vs 8 K (head); parity of 16 K, then interleaved A/B at config 4
set -e
O=gpurun_out/r4chunk; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_chunk16k.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_fullsize.py > $O/tests_chunk16k.log 2>&1
for i in 1 2 3; do
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_head.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_head_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_chunk16k.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_chunk16k_$i.json 2>>$O/err.log
done
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_chunk16k.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof16k -o run -- python bench.py --no-cpu-baseline --no-spread --steps 5 > $O/prof16k.log 2>&1
