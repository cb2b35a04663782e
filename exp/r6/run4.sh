#!/bin/bash
set -e
O=gpurun_out/r6_run4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
bash exp/r6/hostloop.sh a
