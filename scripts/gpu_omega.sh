#!/bin/bash
# over-relaxed dynamics correction passes at the 2-degree bench state (one line each)
set -o pipefail
mkdir -p gpurun_out/omega
export TMPDIR=/tmp
for om in 1.0 1.1 1.2 1.3; do
  timeout -k 10 200 python -u bench.py --no-cpu --newton-seq 0 --steps 2 --dyn-omega $om > gpurun_out/omega/o$om.json 2> gpurun_out/omega/o$om.err \
    || { echo "omega $om FAILED"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/omega/o$om.json').read().strip().splitlines()[-1]); n=d['newton']
print('omega $om', d['value'], n['iters'], n['explicit_rel_res'])"
done
