#!/bin/bash
# IDR(s) against FGMRES at the 2-degree bench state and the coupled C4 state (one line each)
set -o pipefail
mkdir -p gpurun_out/idr
export TMPDIR=/tmp
i=0
while read -r args; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu --newton-seq 0 --steps 2 $args > gpurun_out/idr/v$i.json 2> gpurun_out/idr/v$i.err \
    || { echo "variant $i ($args) FAILED"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/idr/v$i.json').read().strip().splitlines()[-1]); n=d['newton']
print('$args'.ljust(44), d['value'], n.get('iters'), n.get('explicit_rel_res'))"
done <<'LIST'
--solver FGMRES
--solver IDR --idr-s 4
--solver IDR --idr-s 8
--config coupled4 --solver FGMRES
--config coupled4 --solver IDR --idr-s 4
LIST
