#!/bin/bash
# Round 4 first call: the new decode / codec GPU tests, then the driver-shape bench + kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_block_sizes.py tests/test_gpu_codec.py > gpurun_out/r4_first_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_first_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r4_trace.sh
