#!/bin/bash
# code-row shards + full-size dense checks + shard bench + mix ceiling + small-network A/B
set -e
O=gpurun_out/r4b3; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py -k "code_rows or class_rows or (parity and not larger)" > $O/tests_shard.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded_dist.py > $O/tests_dist.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dense_check.py tests/test_gpu_verify.py > $O/tests_dense.log 2>&1
timeout -k 10 300 python bench.py --config cfg5 --sharded --no-spread > $O/cfg5_shard1.json 2> $O/cfg5_shard1.err
for r in 4 5 6 8; do timeout -k 10 60 ./exp/r4/mix_ceiling $r 20 >> $O/mix_ceiling.jsonl; done
for i in 1 2; do
  timeout -k 10 100 python bench.py --config cfg3 --no-cpu-baseline --no-spread > $O/cfg3_base_$i.json
  SAFE_GOSSIP_AMD_SPLIT_BUILD=1 timeout -k 10 100 python bench.py --config cfg3 --no-cpu-baseline --no-spread > $O/cfg3_split_$i.json
  SAFE_GOSSIP_AMD_CONCURRENT_INLISTS=1 timeout -k 10 100 python bench.py --config cfg3 --no-cpu-baseline --no-spread > $O/cfg3_conc_$i.json
done
