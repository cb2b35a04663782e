#!/bin/bash
# timing only (wrong results): config 4's inl_sort without its SibRec writes (random 16-B stores by source id)
set -e
O=gpurun_out/r4nosib; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/head -o run -- python3 bench.py --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_nosib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/nosib -o run -- python3 bench.py --no-cpu-baseline --no-spread > /dev/null 2>>$R/$O/err.log
