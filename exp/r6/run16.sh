#!/bin/bash
# a SEQ harness mismatch seen once at 4c4d258: repeat the case in one
# process with HEAD's library and with GS_RK_ZSKIP_BLK=0 (lib_nozblk.so)
set -e
O=gpurun_out/r6_run16; mkdir -p $O
timeout -k 10 300 python -u exp/r6/seq_repeat.py 20 > $O/head.log 2>&1 || true
tail -n 3 $O/head.log
SAFE_GOSSIP_AMD_LIB=$GRAFT_REPO_ROOT/safe_gossip_amd/lib_nozblk.so timeout -k 10 300 python -u exp/r6/seq_repeat.py 20 > $O/nozblk.log 2>&1 || true
tail -n 3 $O/nozblk.log
