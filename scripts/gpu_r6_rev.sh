#!/bin/bash
# decode emit in descending block order (Infinity Cache reuse of the count pass's last reads): A/B bench, then
# the decode tests on the variant
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in libslatedb_amd.so libslatedb_amd_rev.so; do
    echo "== $lib $i"
    SDB_LIBRARY=$lib timeout -k 10 200 python -u scripts/bench_configs.py --decode --no-granular --reps 20 --cpu-seconds 0 > gpurun_out/rev_$lib.$i.log 2>&1 || exit 1
    grep '^{' gpurun_out/rev_$lib.$i.log | cut -c1-150
  done
done
SDB_LIBRARY=libslatedb_amd_rev.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_failfast.py tests/test_descending.py tests/test_gpu_parity.py tests/test_gpu_block_sizes.py > gpurun_out/rev_tests.log 2>&1; rc=$?; tail -3 gpurun_out/rev_tests.log; exit $rc
