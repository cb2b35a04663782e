#!/bin/bash
# the whole -m gpu suite twice in a row at HEAD (flakiness check after the
# stream-ordering fix)
set -e
O=gpurun_out/r6_run22; mkdir -p $O
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/suite_$i.log 2>&1
  tail -n 1 $O/suite_$i.log
done
