#!/bin/bash
# config 5 DLV sort as a persistent walk over its quarter-bin parts with the next part's region loads in flight (pp: GS_DLV_PP=1) vs HEAD; parity of pp, then interleaved A/B at configs 5 and 2
set -e
O=gpurun_out/r4pp; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pp.so timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_parity.py tests/test_gpu_sharded.py > $O/tests_pp.log 2>&1
for i in 1 2 3; do
  for v in base pp; do
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_${v}_$i.json 2>>$O/err.log
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_${v}_$i.json 2>>$O/err.log
  done
done
