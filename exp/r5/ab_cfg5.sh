#!/bin/bash
# rest of the GPU suite after a failure point, then A/B of config 5 and config 4 (base tree vs HEAD) and the 8-GPU shapes profile
set -e
T=${1:-c}
O=gpurun_out/r5ab_$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_sharded.py tests/test_gpu_sharded_dist.py tests/test_gpu_verify.py tests/test_gpu_wire.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_rest.log 2>&1
timeout -k 10 400 python exp/ab.py --out $O/cfg5 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg5 > $O/ab_cfg5.txt 2>&1
timeout -k 10 300 python exp/ab.py --out $O/cfg2 --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- --config cfg2 > $O/ab_cfg2.txt 2>&1
bash exp/r5/mgpu_prof.sh $T
tail -4 $O/ab_cfg5.txt $O/ab_cfg2.txt
