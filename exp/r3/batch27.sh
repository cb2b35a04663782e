#!/bin/bash
# Round 3 (session 2): per-part DLV tail regions. DLV parity (parity suite,
# full-size partition-build checks), config 2/5 A/B against one shared
# tail counter (exp/lib_sharedtails.so), then SEQ external RPCs (batch 26)
# and the HEAD validation (batch 25).
set -o pipefail
OUT=gpurun_out/r3_batch27
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "dlv or DLV or small or parity_round" > $OUT/tests_dlv.log 2>&1 || { tail -30 $OUT/tests_dlv.log; exit 1; }
tail -1 $OUT/tests_dlv.log
for V in own shared; do
  L=""; [ $V = shared ] && L="SAFE_GOSSIP_AMD_LIB=exp/lib_sharedtails.so"
  for C in cfg2 cfg5; do
    env $L timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline > $OUT/bench_${C}_$V.json 2> $OUT/bench_${C}_$V.err || exit 1
    echo "$V $C $(tail -1 $OUT/bench_${C}_$V.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["spread"])')"
  done
done
bash exp/r3/batch26.sh && bash exp/r3/batch25.sh
