#!/bin/bash
# Kernel trace of rank 0 of an N-rank latitude-band run on one GPU (host transport: one
# process per rank, started here, rank 0 under rocprofv3 --kernel-trace; the in-process rank
# group's threads crashed the tracer twice).  The other ranks share the GPU, so rank 0's
# kernel durations are an upper bound of a rank on its own GPU.
# usage: bash scripts/rank_trace.sh N OUTDIR   (then: python tools/rank_kernels.py OUTDIR/run_results.db STEPS)
N=${1:-8}
OUT=${2:-gpurun_out/rank_trace}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29533} WORLD_SIZE=$N LOCAL_RANK=0
export HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="--gpus $N --transport host --no-cpu --steps 1 --warmup 0 --spmv-reps 0 --cold-reps 0"
pids=()
for r in $(seq 1 $((N - 1))); do
  RANK=$r timeout -k 10 500 python3 -u bench.py $ARGS > $OUT/rank$r.log 2>&1 &
  pids+=($!)
done
RANK=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 -u bench.py $ARGS > $OUT/rank0.json 2> $OUT/rank0.err
rc=$?
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
