#!/bin/bash
# bench.py under a list of environment settings (one per line of $SWEEP_FILE: "VAR=v ... -- args")
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  envs="${line%%--*}"; args="${line#*--}"
  [ "$envs" = "$line" ] && { envs=""; args="$line"; }
  ( for kv in $envs; do export "$kv"; done
    timeout -k 10 240 python -u bench.py --no-cpu --steps 2 --warmup 1 $args > gpurun_out/sweep/env_$i.log 2>&1 ) \
    || { echo "sweep '$line' failed"; tail -5 gpurun_out/sweep/env_$i.log; exit 1; }
  echo "$line :: $(tail -1 gpurun_out/sweep/env_$i.log | python3 -c 'import json,sys; d=json.load(sys.stdin); n=d["newton"]; print(d["value"], n["iters"], n["converged"], n["norm_f1"], n["t_prec_ms"], n["t_solve_ms"])')"
done < "${SWEEP_FILE:-tools/sweep_env.txt}"
echo "sweep ok"
