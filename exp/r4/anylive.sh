#!/bin/bash
# timing only: what the any-live flag's per-block check (a returning load at each block's end) costs the round kernels
set -e
O=gpurun_out/r4any; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd $R
for i in 1 2; do
  for c in cfg4 cfg5; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/${c}_head_$i -o run -- python3 bench.py --config $c --no-cpu-baseline --no-spread > $O/${c}_head_$i.json 2>>$O/err.log
    SAFE_GOSSIP_AMD_LIB=$R/exp/libexp_noany.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/${c}_noany_$i -o run -- python3 bench.py --config $c --no-cpu-baseline --no-spread > $O/${c}_noany_$i.json 2>>$O/err.log
  done
done
