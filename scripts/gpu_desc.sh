#!/bin/bash
# Descending decode in the emit pass: GPU tests, then configs[2] ascending / descending decode with this
# library and with $OLD_LIB (the decoder before the change).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/desc
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_descending.py tests/test_gpu_parity.py tests/test_gpu_block_sizes.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
for L in libslatedb_amd.so ${OLD_LIB:-}; do
  SDB_LIBRARY=$L timeout -k 10 300 python3 scripts/bench_configs.py --decode --no-granular --reps 10 --cpu-seconds 0 > $O/dec_$L.log 2>&1
  rc=$?; echo "== $L"; grep '^{' $O/dec_$L.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
