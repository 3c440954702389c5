#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "natl8 1 2" "natl8 2 2" "gateway16 1 2" "gateway16 3 2" "global4 1 2" "global4 4 2"; do
  timeout -k 10 200 python -u tools/diag_bands.py $a > "gpurun_out/diag_${a// /_}.log" 2>&1 || { echo "diag $a failed"; exit 1; }
done
echo diag ok
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok"
