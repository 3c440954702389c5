#!/bin/bash
# Run the command lines of one section of an indexed call file (argument 1: the file,
# argument 2: the section name; scripts/gpu_calls.txt) on the GPU box one after the other,
# each under its own time limit (a leading "<seconds>|" on the line, default 300).  Output of
# line n goes to gpurun_out/cmds/<section>/<n>.log; a directory that exists already is kept
# and the call writes into <section>.2, .3, ... so no call overwrites the evidence of an
# earlier one.  A limit, abort or crash ends the call (exit code of the step: 124/137 limit,
# 134 abort, 139 segfault); an ordinary failure (exit 1) is reported and the next line runs.
set -o pipefail
file=$1
sec=$2
[ -n "$sec" ] || { echo "usage: gpu_cmds.sh <file> <section>"; exit 2; }
dir=gpurun_out/cmds/$sec
k=2
while [ -e "$dir" ]; do dir=gpurun_out/cmds/$sec.$k; k=$((k + 1)); done
mkdir -p "$dir"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$dir/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
lines=$(awk -v s="[$sec]" '$0 == s {on = 1; next} /^\[/ {on = 0} on && NF && $0 !~ /^#/' "$file")
[ -n "$lines" ] || { echo "no section [$sec] in $file"; exit 2; }
n=0
while IFS= read -r line; do
  n=$((n + 1))
  lim=300
  if [[ $line =~ ^[0-9]+\| ]]; then lim=${line%%|*}; line=${line#*|}; fi
  echo "== $line" > "$dir/$n.log"
  timeout -k 10 $lim bash -c "$line" >> "$dir/$n.log" 2>&1
  rc=$?
  echo "[$n] rc=$rc $line" | tee -a "$dir/summary.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" | tee -a "$dir/summary.txt"; exit $rc; fi
done <<< "$lines"
echo "cmds done ($dir)"
