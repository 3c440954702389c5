#!/bin/bash
# FGMRES steps per decomposition for preconditioner variants (isolating the x-split cost)
set -o pipefail
mkdir -p gpurun_out/decomp
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/decomp/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
CONFIG=gateway16 timeout -k 10 200 python -u scripts/band_iters.py '{"Preconditioner": 1, "FGMRES iterations": 400}' 1,2:1,2:2 > gpurun_out/decomp/d.log 2>&1 && echo d ok || { echo d FAILED; exit 1; }
CONFIG=gateway16 timeout -k 10 200 python -u scripts/band_iters.py '{}' 1,2:1,2:2 > gpurun_out/decomp/e.log 2>&1 && echo e ok || { echo e FAILED; exit 1; }
CONFIG=natl8 timeout -k 10 200 python -u scripts/band_iters.py '{}' 1,2:1,2:2 > gpurun_out/decomp/f.log 2>&1 && echo f ok || { echo f FAILED; exit 1; }
CONFIG=global4 timeout -k 10 200 python -u scripts/band_iters.py '{}' 1,2:1,2:2 > gpurun_out/decomp/g.log 2>&1 && echo g ok || { echo g FAILED; exit 1; }
