#!/bin/bash
# f3 iteration: the device codec tests, then the codec bench (all four codecs, CPU baselines).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/codec
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_codec.py > gpurun_out/codec/tests.log 2>&1
rc=$?; tail -15 gpurun_out/codec/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/bench_configs.py --codec --reps 5 > gpurun_out/codec/bench.log 2>&1
rc=$?; grep "^{" gpurun_out/codec/bench.log | cut -c1-700; tail -3 gpurun_out/codec/bench.log; exit $rc
