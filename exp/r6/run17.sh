#!/bin/bash
# the suite's prefix up to the SEQ harness mismatch seen at 4c4d258, in one
# pytest process: HEAD's library, then GS_RK_ZSKIP_BLK=0 (lib_nozblk.so)
set -e
O=gpurun_out/r6_run17; mkdir -p $O
F="tests/test_gpu_api.py tests/test_gpu_cfg5.py tests/test_gpu_dense_check.py tests/test_gpu_facade.py tests/test_gpu_fullsize.py tests/test_gpu_harness.py"
timeout -k 10 600 python -u -m pytest $F -m gpu -q --timeout 400 --timeout-method thread > $O/head.log 2>&1 || true
tail -n 4 $O/head.log
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/safe_gossip_amd/lib_nozblk.so timeout -k 10 600 python -u -m pytest $F -m gpu -q --timeout 400 --timeout-method thread > $O/nozblk.log 2>&1 || true
tail -n 4 $O/nozblk.log
