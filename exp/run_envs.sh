#!/bin/bash
# A/B timing of environment variants of the production library:
#   run_envs.sh "tag:VAR=v,VAR2=w" ...
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spread > gpurun_out/env_$tag.json 2>gpurun_out/env_$tag.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/env_$tag.json').read().strip().splitlines()[-1]); print('$tag', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms_per_step %.3f'%d['ms_per_step'])"
done
