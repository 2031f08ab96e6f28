#!/bin/bash
# round 6: write-side bench + tests, then a short headline bench (builder selection)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_r6_cz.sh &&
timeout -k 10 400 python -u bench.py --steps 600 --cpu-seconds 4 > gpurun_out/bench_quick.log 2>&1
