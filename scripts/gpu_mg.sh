#!/bin/bash
# One GPU call: preconditioner parity tests (-k $K), band tests, then apply timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${QT:-400} python -u -m pytest tests/test_gpu_parity.py ${EXTRA_TESTS} -m gpu -x -v -s --timeout 120 --timeout-method thread \
    -k "${K:-block_gs or ts_multigrid or dyn_defect or newton_step or bands}" > gpurun_out/pytest_mg.log 2>&1 && echo "tests ok" &&
timeout -k 10 200 python -u scripts/prec_probe.py global2 > gpurun_out/prec_probe.log 2>&1 && echo "probe ok" && cat gpurun_out/prec_probe.log
