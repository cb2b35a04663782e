#!/bin/bash
# run_cfgs.sh "tag|ENV=v,...|bench args" ...
for spec in "$@"; do
  IFS='|' read -r tag envs bargs <<< "$spec"
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py $bargs --no-cpu-baseline --no-spread > gpurun_out/cfg_$tag.json 2>gpurun_out/cfg_$tag.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/cfg_$tag.json').read().strip().splitlines()[-1]); print('$tag', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms_per_step %.3f'%d['ms_per_step'], 'value %.3g'%d['value'])"
done
