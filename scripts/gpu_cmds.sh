#!/bin/bash
# Run the command lines of a file (argument 1) on the GPU box one after the other, each under
# its own time limit (a leading "<seconds>|" on the line, default 300), output into
# gpurun_out/cmds/<n>.log; a limit, abort or crash ends the call, an ordinary failure
# (exit 1) is reported and the next line runs.
set -o pipefail
mkdir -p gpurun_out/cmds
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/cmds/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
n=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  [[ $line == \#* ]] && continue
  n=$((n + 1))
  lim=300
  if [[ $line == *"|"* ]]; then lim=${line%%|*}; line=${line#*|}; fi
  echo "== $line" > gpurun_out/cmds/$n.log
  timeout -k 10 $lim bash -c "$line" >> gpurun_out/cmds/$n.log 2>&1
  rc=$?
  echo "[$n] rc=$rc $line"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done < "$1"
echo "cmds done"
