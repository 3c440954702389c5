#!/bin/bash
# one development iteration on the GPU: selected tests (-k $K), the 2-degree bench line
# (no CPU leg), the preconditioner apply probe, optionally a kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 ${QT:-400} python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${K:-block_gs}" \
    > gpurun_out/pytest_iter.log 2>&1 && echo "tests ok" || { echo "tests FAILED"; tail -30 gpurun_out/pytest_iter.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --newton-seq 0 ${BENCH_ARGS} > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err \
    && echo "bench ok" && cat gpurun_out/bench_iter.json || { echo "bench FAILED"; tail -20 gpurun_out/bench_iter.err; exit 1; }
timeout -k 10 200 python -u scripts/prec_probe.py global2 > gpurun_out/prec_probe.log 2>&1 && cat gpurun_out/prec_probe.log || { echo "probe FAILED"; exit 1; }
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_iter -o run -- \
      python -u bench.py --steps 2 --warmup 1 --no-cpu --newton-seq 0 > gpurun_out/prof_iter.log 2>&1 && echo "prof ok"
fi
