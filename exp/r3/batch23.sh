#!/bin/bash
# Round 3 (session 2): gather-path partition entries as 8-byte records:
# parity (gather path), then configs 3 and 4 A/B against exp/r3/lib_soa2.so;
# and a two-rank gloo rehearsal of bench.py's multi-GPU path on the one GPU.
set -o pipefail
OUT=gpurun_out/r3_batch23
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "not dlv and not partition and not packed" > $OUT/tests_rec.log 2>&1 || { tail -30 $OUT/tests_rec.log; exit 1; }
tail -1 $OUT/tests_rec.log
for i in 1 2 3; do
for V in rec soa2; do
  if [ $V = rec ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  for C in cfg4 cfg3; do
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-spread > $OUT/${C}_${V}_$i.json 2> $OUT/${C}_${V}_$i.err || exit 1
  echo "$C $V $i $(tail -1 $OUT/${C}_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
done
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --config cfg5 --nodes 2000000 --steps 4 --warmup 1 --no-cpu-baseline --no-spread > $OUT/gloo2_cfg5.json 2> $OUT/gloo2_cfg5.err || { tail -20 $OUT/gloo2_cfg5.err; exit 1; }
tail -1 $OUT/gloo2_cfg5.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gloo2 cfg5", d["n_gpus"], d["ms_per_step"], d["config"]["parallelism"][:160])'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_rec -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_rec.log 2>&1 || exit 1
echo done
