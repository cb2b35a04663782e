# Gather calibration + config 5 / config 2 round-kernel profiles
set -o pipefail
mkdir -p gpurun_out/r2d
O=$(pwd)/gpurun_out/r2d
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for m in small wide wide1 stream; do
  timeout -k 10 120 $R/exp/gather_calib $m >> $O/calib_time.jsonl 2>&1 || exit 1
  for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    tag=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/calib_${m}_$tag -o run -- $R/exp/gather_calib $m > /dev/null 2>&1 || exit 1
  done
done
ARGS5="--config cfg5 --steps 8 --warmup 2 --no-cpu-baseline --no-spread"
ARGS2="--config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-spread"
timeout -k 10 300 python3 -u $R/bench.py $ARGS5 > $O/bench_cfg5.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg5_trace -o run -- python3 $R/bench.py $ARGS5 > $O/cfg5_trace.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cfg5_fetch -o run -- python3 $R/bench.py $ARGS5 > $O/cfg5_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cfg5_write -o run -- python3 $R/bench.py $ARGS5 > $O/cfg5_write.log 2>&1 &&
timeout -k 10 300 python3 -u $R/bench.py $ARGS2 > $O/bench_cfg2.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg2_trace -o run -- python3 $R/bench.py $ARGS2 > $O/cfg2_trace.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cfg2_fetch -o run -- python3 $R/bench.py $ARGS2 > $O/cfg2_fetch.log 2>&1
