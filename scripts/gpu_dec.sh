#!/bin/bash
# Decode iteration: decode GPU tests, block-size bench (encode + decode per SstBlockSize), configs[2]
# decode bench and its kernel trace.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/dec
rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_block_sizes.py tests/test_gpu_parity.py tests/test_descending.py tests/test_gpu_configs.py tests/test_gpu_lookup.py ${DEC_K:+-k "$DEC_K"} > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/bench_block_sizes.py > $O/bs.log 2>&1
rc=$?; grep "^{" $O/bs.log; [ $rc -eq 0 ] || { tail -3 $O/bs.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/bench_configs.py --decode --reps 5 --no-granular --cpu-seconds 0 > $O/bench.log 2>&1 < /dev/null
rc=$?; grep "^{" $O/bench.log | cut -c1-400; python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'dec' in r['Name'] or 'desc' in r['Name'] or 'scan' in r['Name']: print(r['Name'][:40], r['Calls'], r['AverageNs'])"; exit $rc
