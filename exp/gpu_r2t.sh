mkdir -p gpurun_out
for c in "2000 1 trickle 0.5 0.2 0.2" "2000 1 trickle 0 0 0" "2000 1 origins 0 0 0" "1030 1 origins 0 0 0" "2000 16 origins 0 0 0" "2000 1 trickle 0.5 0 0" "2000 1 trickle 0 0.2 0.2"; do
echo "== $c" >> gpurun_out/dlv4_debug.log
timeout -k 10 60 python -u exp/dlv4_debug.py $c >> gpurun_out/dlv4_debug.log 2>&1 || exit 1
done
