#!/bin/bash
# round-3 refresh with the current preconditioner: PMC bytes per kernel (2-degree bench
# step and the calibration streams), the coupled C4 line and the 1-degree C5 continuation
# line.  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/r03c/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash scripts/gpu_pmc.sh > gpurun_out/r03c/pmc.log 2>&1 && echo "pmc ok" || { echo "pmc FAILED"; exit 1; }
timeout -k 10 300 python -u bench.py --config coupled4 --steps 5 --warmup 1 > gpurun_out/r03c/bench_coupled4.json 2> gpurun_out/r03c/bench_coupled4.err \
    && echo "c4 bench ok" || { echo "c4 bench FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py --config global1 --mode continuation --steps 1 --warmup 0 > gpurun_out/r03c/bench_global1_cont.json 2> gpurun_out/r03c/bench_global1_cont.err \
    && echo "c5 bench ok" || { echo "c5 bench FAILED"; exit 1; }
