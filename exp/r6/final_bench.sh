#!/bin/bash
# the driver's round-end entry points at HEAD: smoke, then the default bench line
set -e
O=gpurun_out/r6_endcheck; mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -n 1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
grep '^{' $O/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], d['value'], r['frac'], r['traffic'], d['cpu_baseline']['value'], d['build']['id'])"
