#!/bin/bash
# packed DLV round kernel: the own plane words stored to LDS after the metadata, tail and pend loads are issued (stlate) vs base (pendpre); parity of stlate, then interleaved A/B at configs 5 and 2
set -e
O=gpurun_out/r4stlate; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_stlate.so timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_parity.py tests/test_gpu_sharded.py > $O/tests_stlate.log 2>&1
for i in 1 2 3; do
  for v in base stlate; do
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_${v}_$i.json 2>>$O/err.log
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_$v.so timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > $O/cfg2_${v}_$i.json 2>>$O/err.log
  done
done
