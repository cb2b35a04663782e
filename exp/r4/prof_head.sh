#!/bin/bash
# rocprof kernel trace + PMC (FETCH_SIZE, WRITE_SIZE passes) of the bench workloads of configs 4 and 5 at HEAD
set -e
bash profiles/rocprof_r2.sh r4_cfg4
bash profiles/rocprof_r2.sh r4_cfg5 --config cfg5
