#!/bin/bash
# Host cost of the multi-GPU round loop: one RCCL rank, small networks (GPU
# work per round ~0.1 ms, so ms/round shows the loop), the C++ loop
# (gs_net, examples/net_rounds --time) against the Python drivers (bench.py
# --sharded).  Usage: hostloop.sh <tag>
set -e
T=${1:-h}
O=gpurun_out/r6hl_$T; mkdir -p $O
for shape in "1048576 16" "2097152 256"; do
  set -- $shape
  for m in shards slices; do
    timeout -k 10 120 examples/net_rounds --mode $m --transport rccl --world 1 --parts 4 --nodes $1 --rumors $2 --time 50 >> $O/c.jsonl 2>> $O/err.log
  done
  timeout -k 10 200 python bench.py --sharded --mode nodes --parts 4 --nodes $1 --rumors $2 --steps 50 --warmup 3 --no-cpu-baseline --no-spread --pmc off >> $O/py.jsonl 2>> $O/err.log
  timeout -k 10 200 python bench.py --sharded --mode slices --nodes $1 --rumors $2 --steps 50 --warmup 3 --no-cpu-baseline --no-spread --pmc off >> $O/py.jsonl 2>> $O/err.log
done
cat $O/c.jsonl
