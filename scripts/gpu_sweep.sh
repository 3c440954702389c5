#!/bin/bash
# Preconditioner-parameter sweep of the Newton-step bench (one GPU call): each line of
# $SWEEP (or the file $SWEEP_FILE) is a set of bench.py flags; results go to gpurun_out/sweep/<n>.json.
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
n=0
while IFS= read -r flags; do
  [ -z "$flags" ] && continue
  n=$((n+1))
  echo "$flags" > gpurun_out/sweep/$n.flags
  timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --newton-seq 0 $flags \
      > gpurun_out/sweep/$n.json 2> gpurun_out/sweep/$n.err || { echo "sweep $n failed: $flags"; exit 1; }
done <<< "${SWEEP:-$(cat ${SWEEP_FILE:-/dev/null})}"
echo "sweep ok ($n runs)"
