#!/bin/bash
# round-3 measurements in one call: C4 / C5 bench lines, the 2-degree bench line and
# preconditioner apply time, FGMRES steps and communication per decomposition
set -o pipefail
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/r03b/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
true || timeout -k 10 300 python -u bench.py --no-cpu --newton-seq 0 > gpurun_out/r03b/bench_global2.json 2> gpurun_out/r03b/bench_global2.err \
    && echo "g2 bench ok" || { echo "g2 bench FAILED"; exit 1; }
true || timeout -k 10 200 python -u scripts/prec_probe.py global2 > gpurun_out/r03b/prec_probe.log 2>&1 && echo "probe ok" || { echo "probe FAILED"; exit 1; }
true || timeout -k 10 300 python -u bench.py --config coupled4 --steps 5 --warmup 1 > gpurun_out/r03b/bench_coupled4.json 2> gpurun_out/r03b/bench_coupled4.err \
    && echo "c4 bench ok" || { echo "c4 bench FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py --config global1 --mode continuation --steps 1 --warmup 0 > gpurun_out/r03b/bench_global1_cont.json 2> gpurun_out/r03b/bench_global1_cont.err \
    && echo "c5 bench ok" || { echo "c5 bench FAILED"; exit 1; }
timeout -k 10 400 python -u scripts/band_iters.py '{}' 1,2:1,4:1,4,8:1,8 > gpurun_out/r03b/decomp_iters.log 2>&1 && echo "decomp ok" || { echo "decomp FAILED"; exit 1; }
