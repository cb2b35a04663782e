ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="--config cfg5 --steps 3 --warmup 1 --no-cpu-baseline --no-spread"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $ROOT/gpurun_out/pmc_x_sq -o run -- python3 $ROOT/bench.py $B > $ROOT/gpurun_out/pmc_x_sq.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/pmc_x_f -o run -- python3 $ROOT/bench.py $B > $ROOT/gpurun_out/pmc_x_f.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/pmc_x_w -o run -- python3 $ROOT/bench.py $B > $ROOT/gpurun_out/pmc_x_w.log 2>&1 || exit 1
