#!/bin/bash
# run_libcfgs.sh "tag|lib|bench args" ...  (lib = exp/lib_<lib>.so)
for spec in "$@"; do
  IFS='|' read -r tag lib bargs <<< "$spec"
  SAFE_GOSSIP_AMD_LIB=$PWD/exp/lib_$lib.so timeout -k 10 200 python bench.py $bargs --no-cpu-baseline --no-spread > gpurun_out/lc_$tag.json 2>gpurun_out/lc_$tag.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/lc_$tag.json').read().strip().splitlines()[-1]); print('$tag', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms_per_step %.3f'%d['ms_per_step'], 'value %.3g'%d['value'])"
done
