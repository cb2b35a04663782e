#!/bin/bash
# A/B timing of experiment builds (exp/lib_<v>.so) on the default workload.
for v in "$@"; do
  SAFE_GOSSIP_AMD_LIB=$PWD/exp/lib_$v.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spread > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/var_$v.json').read().strip().splitlines()[-1]); print('$v', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms_per_step %.3f'%d['ms_per_step'], 'frac %.3f'%d['roofline']['frac'])"
done
