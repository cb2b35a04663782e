#!/bin/bash
# round-4 baseline at HEAD: configs 4 and 5, one RCCL node-shard rank at config 5
set -e
mkdir -p gpurun_out/r4base
timeout -k 10 200 python bench.py --no-cpu-baseline --no-spread > gpurun_out/r4base/cfg4.json
timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-spread > gpurun_out/r4base/cfg5.json
timeout -k 10 300 python bench.py --config cfg5 --sharded --no-spread > gpurun_out/r4base/cfg5_shard1.json 2> gpurun_out/r4base/cfg5_shard1.err
timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-spread > gpurun_out/r4base/cfg2.json
timeout -k 10 200 python bench.py --config cfg3 --no-cpu-baseline --no-spread > gpurun_out/r4base/cfg3.json
