#!/bin/bash
# one RCCL rank at config 5 with 1/2/4 parts; serialized kernel profile of the 4-part run
set -e
O=gpurun_out/r4b5; mkdir -p $O
for p in 1 2 4; do timeout -k 10 300 python bench.py --config cfg5 --sharded --parts $p --no-spread > $O/cfg5_shard1_p$p.json 2>> $O/err.log; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ser -o run -- python3 bench.py --config cfg5 --sharded --no-spread --no-cpu-baseline --steps 8 > $O/ser.json 2>> $O/err.log
