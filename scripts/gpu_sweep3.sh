#!/bin/bash
# bench variants of the solver parameters (one line each) at the 2-degree bench state
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
i=0
while read -r args; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --no-cpu --newton-seq 0 --steps 2 $args > gpurun_out/sweep/v$i.json 2> gpurun_out/sweep/v$i.err \
    || { echo "variant $i ($args) FAILED"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/sweep/v$i.json').read().strip().splitlines()[-1]); n=d['newton']
print('$args'.ljust(40), d['value'], n['iters'], round(n['t_solve_prec_ms'],1), round(n['t_solve_orth_ms'],1))"
done <<'LIST'
--dyn-iters 4
--dyn-iters 3
--dyn-iters 3 --dyn-omega 1.0
--dyn-iters 5
--dyn-iters 4 --dyn-omega 1.0
--dyn-iters 4 --dyn-mr
--krylov 75
--krylov 110
LIST
