#!/bin/bash
# PMC passes for bench_data/pmc_<tag>.json (tools/pmc_table.py): one counter group per run,
# kernel-trace only, no other trace domains.  Calibration streams of known size, then the
# in-solve counters of every kernel of one benchmark Newton step (FETCH_SIZE and WRITE_SIZE
# in separate runs) and a kernel-trace pass of the same command for the launch times.
# Each pass has its own hard time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/calib_$ctr -o run \
      -- ./scripts/_build/pmc_calib > gpurun_out/pmc/calib_$ctr.log 2>&1 || { echo "calib $ctr failed"; exit 1; }
done
echo "calib ok"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/bench_$ctr -o run \
      -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --newton-seq 0 --no-stream > gpurun_out/pmc/bench_$ctr.log 2>&1 || { echo "bench $ctr failed"; exit 1; }
done
echo "bench pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/bench_trace -o run \
    -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --newton-seq 0 --no-stream > gpurun_out/pmc/bench_trace.log 2>&1 \
    || { echo "bench trace failed"; exit 1; }
echo "bench trace ok"
