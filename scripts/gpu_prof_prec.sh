#!/bin/bash
# rocprofv3 kernel trace of the preconditioner apply probe (50 applies at the bench state)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pprof -o run -- \
    python3 -u scripts/prec_probe.py ${CFG:-global2} > gpurun_out/pprof.log 2>&1 && echo "prof ok" && tail -3 gpurun_out/pprof.log
