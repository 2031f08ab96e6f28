#!/bin/bash
# Decode change check: decode GPU tests, configs[2] (ascending / descending), decode at every block size.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/decchk
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_block_sizes.py tests/test_descending.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_compaction.py tests/test_gpu_codec.py tests/test_gpu_lookup.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_configs.py --decode --reps 10 --cpu-seconds 0 > $O/dec.log 2>&1
rc=$?; grep '^{' $O/dec.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_block_sizes.py > $O/bs.log 2>&1
rc=$?; grep '^{' $O/bs.log | cut -c1-200; exit $rc
