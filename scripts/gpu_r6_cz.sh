#!/bin/bash
# round 6: the f3 write side (compressing codecs) — the bench line first (it checks its own round trips),
# then the write-side tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_configs.py --compress --reps 8 > gpurun_out/cz_bench.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_codec_write.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/cz_test.log 2>&1
