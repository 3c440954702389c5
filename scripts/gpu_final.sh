#!/bin/bash
# Round-end measurement in one GPU call: the default bench line (with the timed CPU
# baseline), its rocprofv3 kernel trace, the 1-degree line and the PMC byte passes.
# Results under gpurun_out/final; copy what is judged into profiles/ (tools/*.py).
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/final/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err \
    && echo "bench ok" || { echo "bench FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run -- \
    python3 -u bench.py --steps 1 --warmup 1 --no-cpu --newton-seq 0 > gpurun_out/final/prof.log 2>&1 \
    && echo "prof ok" || { echo "prof FAILED"; exit 1; }
timeout -k 10 400 python -u bench.py --config global1 --steps 1 --warmup 1 --no-cpu --newton-seq 0 \
    > gpurun_out/final/bench_global1.json 2> gpurun_out/final/bench_global1.err \
    && echo "global1 ok" || { echo "global1 FAILED"; exit 1; }
if [ -n "$PMC" ]; then
  bash scripts/gpu_pmc.sh && echo "pmc ok" || { echo "pmc FAILED"; exit 1; }
fi
