#!/bin/bash
# Round 3 (session 2): DLV partition entries as 12-byte records (one store
# stream per run instead of three arrays): DLV parity, then config-5 A/B
# against the array layout (exp/r3/lib_soa.so) and a kernel trace.
set -o pipefail
OUT=gpurun_out/r3_batch22
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_fullsize.py tests/test_gpu_cfg5.py -m gpu -k "partition or dlv or config5" > $OUT/tests_aos.log 2>&1 || { tail -30 $OUT/tests_aos.log; exit 1; }
tail -1 $OUT/tests_aos.log
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_sliced.py -m gpu -k "dlv or DLV or small or slice or round_parity" > $OUT/tests_parity.log 2>&1 || { tail -30 $OUT/tests_parity.log; exit 1; }
tail -1 $OUT/tests_parity.log
for i in 1 2 3; do
for V in aos soa; do
  if [ $V = aos ]; then L=safe_gossip_amd/libsafe_gossip_amd.so; else L=exp/r3/lib_$V.so; fi
  SAFE_GOSSIP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-spread > $OUT/cfg5_${V}_$i.json 2> $OUT/cfg5_${V}_$i.err || exit 1
  echo "cfg5 $V $i $(tail -1 $OUT/cfg5_${V}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
SAFE_GOSSIP_AMD_LIB=safe_gossip_amd/libsafe_gossip_amd.so timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline --no-spread > $OUT/cfg2_aos_$i.json 2> $OUT/cfg2_aos_$i.err || exit 1
SAFE_GOSSIP_AMD_LIB=exp/r3/lib_soa.so timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline --no-spread > $OUT/cfg2_soa_$i.json 2> $OUT/cfg2_soa_$i.err || exit 1
echo "cfg2 aos/soa $i $(tail -1 $OUT/cfg2_aos_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') $(tail -1 $OUT/cfg2_soa_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_aos -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread > $GRAFT_REPO_ROOT/$OUT/trace_aos.log 2>&1 || exit 1
echo done
