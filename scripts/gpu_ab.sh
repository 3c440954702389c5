#!/bin/bash
# A/B run of library variants on one box (scripts/ab_build.sh, scripts/ab_probe.py): each
# variant under a rocprofv3 kernel trace (AB_TRACE=0: untraced), its own time limit; the first failure ends it.
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
  prof="rocprofv3 --kernel-trace --stats -d gpurun_out/ab/${n}_$v -o run --"
  [ "${AB_TRACE:-1}" = 0 ] && prof=""   # untraced: the tracer slows every launch
  IEMIC_LIB=$lib timeout -k 10 ${AT:-240} $prof \
      python3 -u scripts/ab_probe.py $v ${NSTEP:-3} > gpurun_out/ab/${n}_$v.json 2> gpurun_out/ab/${n}_$v.err \
      && echo "$v ok" || { echo "$v FAILED"; exit 1; }
  db=$(ls gpurun_out/ab/${n}_$v/*/run_results.db gpurun_out/ab/${n}_$v/run_results.db 2>/dev/null | head -1)
  [ -n "$db" ] && python3 tools/rocpd_summary.py "$db" > gpurun_out/ab/${n}_$v.md \
      && python3 tools/gaps.py "$db" 40 > gpurun_out/ab/${n}_$v.gaps.md && rm -rf gpurun_out/ab/${n}_$v
done
echo "ab ok"
