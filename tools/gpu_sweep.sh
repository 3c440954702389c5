#!/bin/bash
# Restart-length / solver-option sweep of bench.py (one GPU); each run has its own limit.
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 240 python -u bench.py --no-cpu --steps 2 --warmup 1 $args > gpurun_out/sweep/run_$i.log 2>&1 \
    || { echo "sweep '$args' failed"; exit 1; }
  echo "$args :: $(tail -1 gpurun_out/sweep/run_$i.log | python3 -c 'import json,sys; d=json.load(sys.stdin); n=d["newton"]; print(d["value"], n["iters"], n["converged"], n["t_prec_ms"], n["t_solve_ms"], n["t_solve_prec_ms"], n["t_solve_orth_ms"], d["roofline"]["launch_us"])')"
done < "${SWEEP_FILE:-tools/sweep.txt}"
echo "sweep ok"
