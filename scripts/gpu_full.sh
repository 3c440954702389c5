#!/bin/bash
# Full GPU suite, bench, rocprofv3 kernel trace of one bench step (every step time-limited,
# chained with &&, so the first failure ends the call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
rm -rf gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 && echo "bench ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu --newton-seq 0 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 && echo "prof ok"
