#!/bin/bash
# Round 3 (session 2): the DLV build's first partition fused into the
# transition launch (gs_dlv4.hip epilogue, no dl_coarse launch): DLV parity
# (partition builds vs the gather path, config-5 laws, slices), then config-5
# A/B against SAFE_GOSSIP_AMD_FUSE_COARSE=0.
set -o pipefail
OUT=gpurun_out/r3_batch20
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
SAFE_GOSSIP_AMD_DEBUG=1 timeout -k 10 600 $T tests/test_gpu_fullsize.py tests/test_gpu_cfg5.py -m gpu -k "partition or dlv or config5" > $OUT/tests_fused.log 2>&1 || { grep -a "safe_gossip_amd:" $OUT/tests_fused.log | head -3; tail -30 $OUT/tests_fused.log; exit 1; }
tail -1 $OUT/tests_fused.log
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_sliced.py tests/test_gpu_api.py -m gpu > $OUT/tests_parity.log 2>&1 || { tail -30 $OUT/tests_parity.log; exit 1; }
tail -1 $OUT/tests_parity.log
for i in 1 2 3; do
for V in fused split; do
  F=1; if [ $V = split ]; then F=0; fi
  SAFE_GOSSIP_AMD_FUSE_COARSE=$F timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_fused -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_fused.log 2>&1 || exit 1
echo done
