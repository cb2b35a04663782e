#!/bin/bash
# shard round kernel: missing pushers' rows branched around (lib_shbr.so,
# (rejected: 0.3045 -> 0.320 ms per shard launch; the knob was removed, profiles/r6/rejected_shard_branch/)
# GS_RK_SHARD_BRANCH=1) vs loaded from row 0: shard parity tests on the
# variant, then config 4's 8-shard shape interleaved (kernels serialised)
set -e
O=gpurun_out/r6_run21; mkdir -p $O
R=$GRAFT_REPO_ROOT
SAFE_GOSSIP_AMD_LIB=$R/safe_gossip_amd/lib_shbr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_net.py tests/test_gpu_reuse.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -n 2 $O/tests.log
cd /tmp && export TMPDIR=/tmp && cd $R
for i in 1 2; do
  for v in head shbr; do
    L=$R/safe_gossip_amd/libsafe_gossip_amd.so; [ $v = shbr ] && L=$R/safe_gossip_amd/lib_shbr.so
    SAFE_GOSSIP_AMD_LIB=$L AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${v}_$i -o run -- python3 exp/shard_prof.py 8 30 1 > $O/${v}_$i.txt 2>&1
    grep -h "round_kernel<false, 1, true" $R/$O/${v}_$i/run_kernel_stats.csv | cut -d, -f1-4
  done
done
