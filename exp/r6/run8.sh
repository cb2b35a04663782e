#!/bin/bash
set -e
O=gpurun_out/r6_run8; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sliced.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
bash exp/r6/shapes.sh a
