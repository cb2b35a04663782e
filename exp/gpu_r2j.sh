set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_sparse.log
: > $out
for rep in 1 2; do
SAFE_GOSSIP_AMD_LIB=exp/lib_head.so timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 head >> $out 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=dense timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 new >> $out 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=auto timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 new >> $out 2>&1 &&
SAFE_GOSSIP_AMD_SPARSE=on timeout -k 10 120 python -u exp/ab_sparse.py 16777216 256 20 new >> $out 2>&1 || exit 1
done
