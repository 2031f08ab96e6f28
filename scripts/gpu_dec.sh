#!/bin/bash
# Decode iteration: decode GPU tests, configs[2] decode bench, rocprof kernel stats of the decode.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; rm -rf gpurun_out/decprof
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_descending.py tests/test_gpu_configs.py tests/test_gpu_lookup.py -k "${DEC_K:-decode or desc or configs2 or lookup}" > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dec_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/dec_tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/bench_configs.py --decode --reps 10 > gpurun_out/dec_bench.log 2>&1
rc=$?; grep "^{" gpurun_out/dec_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/decprof -o run --output-format csv -- python3 scripts/bench_configs.py --decode --reps 5 --no-granular > gpurun_out/decprof.log 2>&1
rc=$?; cut -d, -f1-4 gpurun_out/decprof/run_kernel_stats.csv | grep -E "k_dec|scan" ; exit $rc
