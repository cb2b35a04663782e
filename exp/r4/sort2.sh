#!/bin/bash
# config 4 in-list sort: live tag carried in the id register (ltag: inl_sort<0> 108 -> 88 VGPRs) and, on top, half-bin sorts of own regions with two 1024-thread blocks per CU (sort2: GS_SORT_SPLIT_LOG=1, GS_SORT_MINW_SPLIT=8, 64 VGPRs, 9 spilled) vs head; parity of both, then interleaved A/B at config 4
set -e
O=gpurun_out/r4sort2; mkdir -p $O
R=$GRAFT_REPO_ROOT
for v in ltag sort2; do
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $O/tests_$v.log 2>&1
done
for i in 1 2 3; do
  for v in head ltag sort2; do
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > $O/cfg4_${v}_$i.json 2>>$O/err.log
  done
done
