#!/bin/bash
set -e
O=gpurun_out/r6_run11; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
timeout -k 10 300 python bench.py --gpus 3 --dist-backend gloo --nodes 200000 --rumors 64 --steps 10 > $O/gloo3.json 2> $O/gloo3.err
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --nodes 300000 --rumors 16 --config cfg5 --steps 10 > $O/gloo2_cfg5.json 2> $O/gloo2_cfg5.err
grep -h '^{' $O/gloo*.json | cut -c1-200
