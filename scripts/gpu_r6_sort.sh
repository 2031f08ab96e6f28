#!/bin/bash
# standalone bloom (configs[3]): k_bloom_sort6 (rank reservations in flight together) vs the previous build; tests
set -u
export TMPDIR=/tmp
O=gpurun_out/sort
rm -rf $O; mkdir -p $O
for i in 1 2; do
for lib in libslatedb_amd_old.so libslatedb_amd.so; do
  SDB_LIBRARY=$lib timeout -k 10 200 python3 scripts/bench_configs.py --bloom --reps 40 > $O/b_$lib.$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  echo "$lib $(grep '"bloom configs\[3\]"' $O/b_$lib.$i.log | cut -c1-200)"
done
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 20 > $O/t.log 2>&1 || { echo "trace rc=$?"; exit 1; }
grep -E 'k_bloom' $O/t/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/e -o run --output-format csv -- python3 bench.py --streams 1 --steps 40 --warmup 5 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/e.log 2>&1 || { echo "trace rc=$?"; exit 1; }
grep -E 'k_facts|k_seg|k_emit<' $O/e/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_prefix.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; exit $rc
