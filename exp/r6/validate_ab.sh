#!/bin/bash
# Round 6: whole -m gpu suite + smoke, then an interleaved A/B of the tree
# against exp/base_tree (HEAD before the change).  Usage: validate_ab.sh <tag> [bench args...]
set -e
T=${1:-v}; shift || true
O=gpurun_out/r6_$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -n 2 $O/gpu_tests.log
timeout -k 10 600 python exp/ab.py --out $O/ab --reps 3 --variant "base:dir=exp/base_tree" --variant "head:dir=." -- "$@" > $O/ab.log 2>&1
tail -n 3 $O/ab.log
