#!/bin/bash
# Round 3 (session 2): external RPCs under the SEQ schedule (wire tests vs the
# oracle), the SEQ parity suite, and the GPU suite's wire/API files.
set -o pipefail
OUT=gpurun_out/r3_batch26
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_wire.py tests/test_gpu_api.py tests/test_gpu_verify.py -m gpu > $OUT/tests_wire.log 2>&1 || { tail -40 $OUT/tests_wire.log; exit 1; }
tail -1 $OUT/tests_wire.log
timeout -k 10 600 $T tests/test_gpu_parity.py -m gpu -k "seq or SEQ" > $OUT/tests_seq.log 2>&1 || { tail -30 $OUT/tests_seq.log; exit 1; }
tail -1 $OUT/tests_seq.log
echo done
