#!/bin/bash
# early T/S (side-stream V-cycles) parity tests, apply timing and bench step time per ts_at
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "block_gs_early or block_gs_default" > gpurun_out/pytest_tsat.log 2>&1 && echo "tests ok" &&
timeout -k 10 200 python -u scripts/prec_probe.py global2 "" "TS after dyn pass=2" "TS after dyn pass=3" > gpurun_out/probe_tsat.log 2>&1 && cat gpurun_out/probe_tsat.log &&
for t in 0 3 2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --ts-at $t > gpurun_out/bench_tsat$t.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_tsat$t.log').read().strip().splitlines()[-1]); print($t, d['value'], d['newton']['iters'], d['newton']['t_solve_prec_ms'])"
done
