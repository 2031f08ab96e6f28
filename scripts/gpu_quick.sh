#!/bin/bash
# Quick GPU iteration: full -m gpu suite, then the bench (no CPU leg).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/q_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/q_tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-600} --warmup 10 --no-cpu ${BENCH_ARGS:-} > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err
rc=$?; python3 -c "
import json; d=json.load(open('gpurun_out/q_bench.json')); r=d['roofline']
print('value', d['value'], 'ms/SST', r['device_ms_per_sst'], 'frac', r['frac'], 'emit', r['k_emit']['frac'], 'single', d['single_sst'])
print({k: round(v/8*1000,1) for k,v in r['stage_ms_per_step'].items()})" ; tail -2 gpurun_out/q_bench.err; exit $rc
