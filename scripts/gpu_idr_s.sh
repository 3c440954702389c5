#!/bin/bash
# IDR(s) shadow-space size at the 2-degree bench state (one line each)
set -o pipefail
mkdir -p gpurun_out/idrs
export TMPDIR=/tmp
for s in 2 3 4 5 6; do
  timeout -k 10 300 python -u bench.py --no-cpu --newton-seq 0 --steps 2 --solver IDR --idr-s $s > gpurun_out/idrs/s$s.json 2> gpurun_out/idrs/s$s.err \
    || { echo "IDR($s) FAILED"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/idrs/s$s.json').read().strip().splitlines()[-1]); n=d['newton']
print('IDR($s)', d['value'], n.get('iters'), n.get('explicit_rel_res'))"
done
