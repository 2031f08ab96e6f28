#!/bin/bash
# probe + rocprofv3 kernel stats of the bench + bench variants.  Stops at the first crash.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${PROBE:-}" ]; then
  timeout -k 10 120 ./scripts/probe > gpurun_out/probe.log 2>&1; rc=$?; echo "probe rc=$rc"; cat gpurun_out/probe.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --bpk 0 > gpurun_out/bench_nobloom.log 2>&1
rc=$?; echo "bench bpk0 rc=$rc"; tail -1 gpurun_out/bench_nobloom.log | cut -c1-200
exit $rc
