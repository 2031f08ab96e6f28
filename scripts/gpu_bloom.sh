#!/bin/bash
# Bloom iteration: bloom GPU tests, configs[3] bench, kernel trace + FETCH/WRITE passes of configs[3].
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/bloom
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "bloom or configs3" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 20 > $O/bench.log 2>&1
rc=$?; grep '^{' $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cut -d, -f1-4 $O/trace/run_kernel_stats.csv | grep bloom
for c in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC:-}; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 3 > $O/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_kernels.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE
