#!/bin/bash
# Iteration call: GPU tests ($TESTS, default all), the bench without CPU leg, bloom kernel trace.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/iter
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 600 --warmup 10 --no-cpu > $O/bench.json 2> $O/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; b=d['config']['ssts_per_gpu_per_step']
print('value', d['value'], 'us/SST', round(r['device_ms_per_sst']*1000,2), 'frac', r['frac'], 'one_stream', d['one_stream']['device_ms_per_sst'], 'single', d['single_sst']['device_ms_per_sst'])
print({k: round(v/b*1000,2) for k,v in r['stage_ms_per_step'].items()})"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/bloom -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 20 > $O/bloom.log 2>&1
rc=$?; grep '^{' $O/bloom.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
python3 -c "
import csv
for r in csv.DictReader(open('$O/bloom/run_kernel_stats.csv')): print(r['Name'][:40], r['AverageNs'])"
