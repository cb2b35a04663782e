#!/bin/bash
# 8-rank rehearsal of the driver's N=8 bench run on ONE GPU: gloo (host-staged
# exchanges), both multi-GPU modes, default steps/warmup and the spread run;
# wall time per config.  Usage: rehearse8.sh <tag> [configs...]
set -e
T=${1:-a}; shift || true
O=gpurun_out/r5r8_$T; mkdir -p $O
for c in ${@:-cfg4 cfg5}; do
  s=$(date +%s.%N)
  timeout -k 10 900 python bench.py --gpus 8 --dist-backend gloo --config $c > $O/$c.json 2> $O/$c.err
  e=$(date +%s.%N)
  python -c "print('$c wall_s', round($e - $s, 1))" | tee -a $O/wall.txt
done
