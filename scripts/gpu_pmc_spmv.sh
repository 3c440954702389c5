#!/bin/bash
# PMC bytes of the in-solve SpMV alone (tools/pmc_report.py layout): calibration streams,
# then FETCH_SIZE and WRITE_SIZE of k_spmv7c over one benchmark Newton step (kernel filter,
# one counter group per run) and a kernel-trace pass.  Argument: the output directory under
# gpurun_out/ (the library variant comes from the caller's environment).
set -o pipefail
d=gpurun_out/${1:-pmc_spmv}
mkdir -p $d
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d $d/calib_$ctr -o run \
      -- ./scripts/_build/pmc_calib > $d/calib_$ctr.log 2>&1 || { echo "calib $ctr failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex k_spmv7c --output-format csv -d $d/spmv_$ctr -o run \
      -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --newton-seq 0 --no-stream > $d/spmv_$ctr.log 2>&1 \
      || { echo "spmv $ctr failed"; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --kernel-include-regex k_spmv7c --output-format csv -d $d/spmv_trace -o run \
    -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --newton-seq 0 --no-stream > $d/spmv_trace.log 2>&1 \
    || { echo "spmv trace failed"; exit 1; }
python3 tools/pmc_report.py $d global2 > $d/report.json && cat $d/report.json
