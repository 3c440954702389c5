#!/bin/bash
# Round-end check in one GPU call: the GPU test suite, smoke(), the default bench line and
# its rocprofv3 kernel trace.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/round
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/round/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/round/pytest_gpu.log 2>&1 && echo "pytest ok" || { echo "pytest FAILED"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 \
    && echo "smoke ok" || { echo "smoke FAILED"; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/round/bench.json 2> gpurun_out/round/bench.err \
    && echo "bench ok" || { echo "bench FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/round/prof -o run -- \
    python3 -u bench.py --steps 1 --warmup 1 --no-cpu --newton-seq 0 > gpurun_out/round/prof.log 2>&1 \
    && echo "prof ok" || { echo "prof FAILED"; exit 1; }
