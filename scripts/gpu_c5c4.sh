#!/bin/bash
# configs C5 / C4: the 1-degree continuation-step test and bench line, the coupled bench
# line from its branch state (outputs under gpurun_out/c5c4)
set -o pipefail
mkdir -p gpurun_out/c5c4
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/c5c4/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
true || timeout -k 10 300 python -u -m pytest tests/test_gpu_reference_tests.py -x -v -s --timeout 280 --timeout-method thread -k global1 \
    > gpurun_out/c5c4/pytest_c5.log 2>&1 && echo "c5 test ok" || { echo "c5 test FAILED"; exit 1; }
timeout -k 10 300 python -u bench.py --config coupled4 --steps 5 --warmup 1 > gpurun_out/c5c4/bench_coupled4.json 2> gpurun_out/c5c4/bench_coupled4.err \
    && echo "c4 bench ok" || { echo "c4 bench FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py --config global1 --mode continuation --steps 1 --warmup 0 > gpurun_out/c5c4/bench_global1_cont.json 2> gpurun_out/c5c4/bench_global1_cont.err \
    && echo "c5 bench ok" || { echo "c5 bench FAILED"; exit 1; }
