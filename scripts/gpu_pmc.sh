#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only, no other trace domains):
# calibration streams of known size, then the cold-cache SpMV probe.  Each pass has its
# own hard time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CFG=${CFG:-global2}
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/calib_$ctr -o run \
      -- ./scripts/_build/pmc_calib > gpurun_out/pmc/calib_$ctr.log 2>&1 || { echo "calib $ctr failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/spmv_$ctr -o run \
      -- python3 -u scripts/spmv_probe.py $CFG 5 > gpurun_out/pmc/spmv_$ctr.log 2>&1 || { echo "spmv $ctr failed"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/spmv_trace -o run \
    -- python3 -u scripts/spmv_probe.py $CFG 5 > gpurun_out/pmc/spmv_trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo "pmc ok"
# in-solve counters of every kernel of one benchmark Newton step (warm caches, as timed)
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/bench_$ctr -o run \
      -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --newton-seq 0 > gpurun_out/pmc/bench_$ctr.log 2>&1 || { echo "bench $ctr failed"; exit 1; }
done
echo "bench pmc ok"
