#!/bin/bash
# code rows with targets (no ids, DLV build over received rows): parity, full-size check, bench, per-shard profile
set -e
O=gpurun_out/r4b4; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py > $O/tests_shard.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --durations=0 --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py -k "config5 or small" > $O/tests_dense.log 2>&1
timeout -k 10 300 python bench.py --config cfg5 --sharded --no-spread > $O/cfg5_shard1.json 2> $O/cfg5_shard1.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg5_8 -o run -- python3 exp/shard_prof.py 8 8 3 cfg5 > $O/cfg5_8.txt 2>&1
