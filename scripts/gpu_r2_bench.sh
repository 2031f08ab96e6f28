#!/bin/bash
# Round-2 bench + rocprof kernel stats of the same command (no PMC here).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps ${STEPS:-1500} --warmup 20 ${BENCH_ARGS:---no-cpu} > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err
rc=$?; cat gpurun_out/r2_bench.json; tail -3 gpurun_out/r2_bench.err; [ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof -o run -- python3 bench.py --steps 200 --warmup 5 --no-cpu --single-steps 0 --stage-steps 0 > gpurun_out/r2_prof.log 2>&1
  rc=$?; tail -3 gpurun_out/r2_prof.log; exit $rc
fi
