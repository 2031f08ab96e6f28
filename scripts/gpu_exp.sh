#!/bin/bash
# Diagnostic builds (wrong output by design): rocprof kernel stats of the decode per build in $EXPS.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for x in ${EXPS}; do
  rm -rf gpurun_out/exp_$x
  SDB_LIBRARY=libslatedb_amd_$x.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/exp_$x -o run --output-format csv -- python3 scripts/bench_configs.py ${EXP_ARGS:---decode --reps 3 --no-granular} > gpurun_out/exp_$x.log 2>&1
  rc=$?; echo "== $x rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  cut -d, -f1-4 gpurun_out/exp_$x/run_kernel_stats.csv | grep -E "${EXP_GREP:-k_dec}"
done
