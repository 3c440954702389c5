#!/bin/bash
# One GPU call: selected tests (-k $K), then optionally the full GPU suite and the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# heartbeat: long single steps (1-degree tests, benches) still write under gpurun_out
( while sleep 45; do date +%T >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 ${QT:-300} python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "${K:-block_gs}" \
    > gpurun_out/pytest_quick.log 2>&1 && echo "quick ok" || { echo "quick FAILED"; exit 1; }
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" || { echo "pytest FAILED"; exit 1; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 && echo "bench ok" || { echo "bench FAILED"; exit 1; }
fi
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
      python -u bench.py --steps 1 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 && echo "prof ok"
fi
if [ -n "$MB" ]; then
  timeout -k 10 120 $MB > gpurun_out/mb.log 2>&1 && echo "mb ok" || { echo "mb FAILED"; exit 1; }
fi
