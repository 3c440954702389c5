#!/bin/bash
# One GPU call of round 4: selected GPU tests (-k $K, per-test limit $TT), then optionally the
# full GPU suite ($FULL), bench lines ($BENCH, $BENCH2: argument strings), a rocprofv3 kernel
# trace of a bench step ($PROF) and a micro-benchmark command ($MB).  Each GPU step has its
# own limit; a limit, abort or crash ends the call (test assertion failures do not).
set -o pipefail
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
( while sleep 45; do date +%T >> gpurun_out/r04/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$K" ]; then
  # test failures (exit 1) do not stop the call; a limit, abort or crash does
  timeout -k 10 ${QT:-400} python -u -m pytest tests -m gpu --maxfail=6 -v -s --timeout ${TT:-120} --timeout-method thread -k "$K" \
      > gpurun_out/r04/pytest_sel.log 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then echo "selected ok"; elif [ $rc -eq 1 ]; then echo "selected: test failures"; else echo "selected FAILED rc=$rc"; exit 1; fi
fi
if [ -n "$FULL" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/r04/pytest_gpu.log 2>&1 && echo "pytest ok" || { echo "pytest FAILED"; exit 1; }
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1 \
      && echo "smoke ok" || { echo "smoke FAILED"; exit 1; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BT:-400} python -u bench.py $BENCH > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err \
      && echo "bench ok" || { echo "bench FAILED"; exit 1; }
fi
if [ -n "$BENCH2" ]; then
  timeout -k 10 ${BT:-400} python -u bench.py $BENCH2 > gpurun_out/r04/bench2.json 2> gpurun_out/r04/bench2.err \
      && echo "bench2 ok" || { echo "bench2 FAILED"; exit 1; }
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/prof -o run -- \
      python3 -u bench.py --steps 1 --warmup 1 --no-cpu --newton-seq 0 $PROF > gpurun_out/r04/prof.log 2>&1 \
      && echo "prof ok" || { echo "prof FAILED"; exit 1; }
fi
if [ -n "$MB" ]; then
  timeout -k 10 ${MT:-200} $MB > gpurun_out/r04/mb.log 2>&1 && echo "mb ok" || { echo "mb FAILED"; exit 1; }
fi
echo "all ok"
