#!/bin/bash
# config 5 packed DLV round kernel: the pend votes of nodes back from offline loaded with the metadata (pendpre) vs head; parity of pendpre (dense check with faults, DLV parity, shards), then interleaved A/B at config 5
set -e
O=gpurun_out/r4pendpre; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pendpre.so timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_parity.py tests/test_gpu_sharded.py > $O/tests_pendpre.log 2>&1
for i in 1 2 3; do
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_head.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_head_$i.json 2>>$O/err.log
  SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_pendpre.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > $O/cfg5_pendpre_$i.json 2>>$O/err.log
done
