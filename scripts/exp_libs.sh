#!/bin/bash
# bench each experiment library (SDB_LIBRARY=...) and print the per-stage times; stops at a crash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/exp
for lib in ${LIBS:-libslatedb_amd.so}; do
  SDB_LIBRARY=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-verify ${BENCH_EXTRA:-} > gpurun_out/exp/$lib.log 2>&1
  rc=$?
  echo "$lib rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/exp/$lib.log | head -1) $(grep -o '"stage_ms": {[^}]*}' gpurun_out/exp/$lib.log)"
  [ $rc -eq 0 ] || exit $rc
done
