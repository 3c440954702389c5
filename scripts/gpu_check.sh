#!/bin/bash
# One GPU call: parity tests, bench, rocprof kernel stats.  Every GPU step has its own
# time limit and the steps are chained with &&, so the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 && echo "bench ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
    python -u bench.py --steps 1 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 && echo "prof ok"
