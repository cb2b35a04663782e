#!/bin/bash
# bench.py --gpus 8 on ONE GPU with 8 gloo ranks: all four modes (the Python
# drivers; the library loop over the host collectives), the spread run, wall
# time.  Usage: rehearse8.sh <tag> [bench args]
set -e
T=${1:-a}; shift || true
O=gpurun_out/r6r8_$T; mkdir -p $O
s=$(date +%s.%N)
timeout -k 10 900 python bench.py --gpus 8 --dist-backend gloo --deadline 840 "$@" > $O/bench8.json 2> $O/bench8.err
e=$(date +%s.%N)
python -c "print('wall_s', round($e - $s, 1))" | tee $O/wall.txt
