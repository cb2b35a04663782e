#!/bin/bash
# Round 3 (session 2): shard row flags (receivers skip rows flagged empty).
# Shard parity (flags on and off), then A/B: bench --sharded (one RCCL rank,
# self-copy exchanges) at configs 4 and 5, and per-kernel times of 8 local
# shards over 30 rounds of config 4 (kernels serialised); then the config 2/3
# kernel traces (batch 28).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r3_batch29
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py -m gpu > $OUT/tests_shard.log 2>&1 || { tail -30 $OUT/tests_shard.log; exit 1; }
tail -1 $OUT/tests_shard.log
for it in 1 2; do
  for F in 1 0; do
    for C in cfg4 cfg5; do
      SAFE_GOSSIP_AMD_SHARD_FLAGS=$F timeout -k 10 400 python -u bench.py --config $C --sharded --no-cpu-baseline --no-spread > $OUT/bench_${C}_f${F}_$it.json 2> $OUT/bench_${C}_f${F}_$it.err || { tail -5 $OUT/bench_${C}_f${F}_$it.err; exit 1; }
      echo "flags=$F $C $(tail -1 $OUT/bench_${C}_f${F}_$it.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for F in 1 0; do
  SAFE_GOSSIP_AMD_SHARD_FLAGS=$F AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shard8_f$F -o run -- python3 $ROOT/exp/shard_prof.py 8 30 0 > $OUT/shard8_f$F.log 2>&1 || { tail -5 $OUT/shard8_f$F.log; exit 1; }
  tail -1 $OUT/shard8_f$F.log
done
cd $ROOT && bash exp/r3/batch28.sh
