#!/bin/bash
# A/B of the SpMV kernel variants (IEMIC_SPMV=1 thread/cell, 2 two cells/thread, 6 wave/row, 7 LDS-staged x)
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for v in ${VARIANTS:-6 7}; do
  IEMIC_SPMV=$v timeout -k 10 120 python3 -u scripts/spmv_probe.py ${CFG:-global2} 20 > gpurun_out/ab/spmv_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/ab/spmv_$v.log)"
done
