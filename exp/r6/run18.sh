#!/bin/bash
# two one-off mismatches at 4c4d258 / ba35ef6: the affected tests repeated in
# one process, HEAD's library, then every all-A store skip off (lib_noskip.so)
set -e
O=gpurun_out/r6_run18; mkdir -p $O
timeout -k 10 400 python -u exp/r6/net_repeat.py 25 > $O/head.log 2>&1 || true
tail -n 3 $O/head.log
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/safe_gossip_amd/lib_noskip.so timeout -k 10 400 python -u exp/r6/net_repeat.py 25 > $O/noskip.log 2>&1 || true
tail -n 3 $O/noskip.log
