set -o pipefail
# Rumor slices at full size (config 4) over 2 and 4 gloo ranks on the box's one GPU: the spread
# record (rounds, first full round, nodes complete) must equal the single-GPU run's; and a
# kernel-trace profile of one slice engine of an 8-GPU run (R/8 = 32 rumors over all 2^24 nodes).
mkdir -p gpurun_out/slices_rehearsal
timeout -k 10 500 python -u bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/slices_rehearsal/bench2_gloo.json 2> gpurun_out/slices_rehearsal/bench2_gloo.err || exit 1
timeout -k 10 600 python -u bench.py --gpus 4 --dist-backend gloo --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/slices_rehearsal/bench4_gloo.json 2> gpurun_out/slices_rehearsal/bench4_gloo.err || exit 1
timeout -k 10 300 bash profiles/rocprof_r2.sh r2_slice_R32 --rumors 32 > gpurun_out/prof_r2_slice_R32.log 2>&1 || exit 1
