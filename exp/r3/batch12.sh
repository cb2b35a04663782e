#!/bin/bash
# Round 3 (session 2): 32-bit lanes where a lane holds one node (R_pad 32,
# the rumor-slice shape of 8 GPUs) and two (R_pad 64, config 3); host enqueue
# cost with fence-free timing events; the quarter-bin DLV variant's launch
# failure; in-list partitions that keep each entry's part (no binary search),
# A/B at configs 4 and 5; SQ counters of the config-5 build kernels.
set -o pipefail
OUT=gpurun_out/r3_batch12
mkdir -p $OUT
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_dsl2.so AMD_LOG_LEVEL=1 timeout -k 10 120 python -u exp/r3/dsl2_diag.py 100000000 > $OUT/dsl2_diag.log 2>&1; echo "dsl2 diag rc=$?"; tail -5 $OUT/dsl2_diag.log
timeout -k 10 200 python -u exp/r3/host_overhead.py > $OUT/host_overhead.jsonl 2> $OUT/host_overhead.err || exit 1
cat $OUT/host_overhead.jsonl
for i in 1 2; do
for E in 1 0; do
  SAFE_GOSSIP_AMD_W32=$E timeout -k 10 200 python -u bench.py --rumors 32 --no-cpu-baseline --no-spread > $OUT/r32_w${E}_$i.json 2> $OUT/r32_w${E}_$i.err || exit 1
  echo "2^24x32 w32=$E $i $(tail -1 $OUT/r32_w${E}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"][:30])')"
  SAFE_GOSSIP_AMD_W32=$E timeout -k 10 200 python -u bench.py --config cfg3 --no-cpu-baseline --no-spread > $OUT/cfg3_w${E}_$i.json 2> $OUT/cfg3_w${E}_$i.err || exit 1
  echo "cfg3 w32=$E $i $(tail -1 $OUT/cfg3_w${E}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"][:30])')"
done
done
for i in 1 2; do
for V in prev head; do
  if [ $V = head ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  for C in cfg4 cfg5; do
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}_${V}_$i.json 2> $OUT/${C}_${V}_$i.err || exit 1
  echo "$C $V $i $(tail -1 $OUT/${C}_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
done
timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline --no-spread > $OUT/cfg2.json 2> $OUT/cfg2.err || exit 1
echo "cfg2 $(tail -1 $OUT/cfg2.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5.json 2> $OUT/cfg5.err || exit 1
echo "cfg5 $(tail -1 $OUT/cfg5.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
cd /tmp && export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
ARGS="--config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $ROOT/$OUT/sq5 -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/sq5.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d $ROOT/$OUT/sq5b -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/sq5b.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/$OUT/fetch5 -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/fetch5.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/$OUT/write5 -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/write5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace5 -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/trace5.log 2>&1 || exit 1
echo done
