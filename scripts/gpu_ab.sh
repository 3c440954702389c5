#!/bin/bash
# A/B run of library variants on one box (scripts/ab_build.sh, scripts/ab_probe.py): each
# variant under a rocprofv3 kernel trace, its own time limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/ab/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
n=0
for v in ${VARIANTS:-base}; do
  n=$((n + 1))
  lib=libiemic_amd_$v.so
  [ "$v" = base ] && lib=libiemic_amd.so
  IEMIC_LIB=$lib timeout -k 10 ${AT:-240} rocprofv3 --kernel-trace --stats -d gpurun_out/ab/${n}_$v -o run -- \
      python3 -u scripts/ab_probe.py $v ${NSTEP:-3} > gpurun_out/ab/${n}_$v.json 2> gpurun_out/ab/${n}_$v.err \
      && echo "$v ok" || { echo "$v FAILED"; exit 1; }
done
echo "ab ok"
