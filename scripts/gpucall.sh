#!/bin/bash
# Submit one gpurun command (argument 1) with limit $LIMIT, waiting out infrastructure-side
# refusals (no free box, backoff, a box lost while being prepared: nothing of the command ran)
# up to $TRIES times.  A call whose command ran is never resubmitted, whatever its outcome.
# Output: gpurun_out/$OUT (default call.txt).
OUT=gpurun_out/${OUT:-call.txt}
for t in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout ${LIMIT:-1200} -- "$1" > $OUT 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|backing off" $OUT && ! grep -q "status=ok\|status=failed\|status=timeout" $OUT; then
    w=$(grep -o "retry in [0-9]*s" $OUT | grep -o "[0-9]*" | head -1)
    sleep $(( ${w:-150} + 20 ))
    continue
  fi
  exit $rc
done
exit 3
