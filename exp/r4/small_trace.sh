#!/bin/bash
# kernel traces of configs 2 and 3 (where a round's time goes on small networks)
set -e
O=gpurun_out/r4small; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd $R
for c in cfg2 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-spread > $O/$c.json 2>>$O/err.log
done
