#!/bin/bash
# Encode change check: encode GPU tests, then the bench on one and two streams with stage times.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/encchk
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_prefix.py tests/test_gpu_block_sizes.py} > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
for st in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 600 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 40 --streams $st > $O/b$st.json 2> $O/b$st.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 $O/b$st.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$O/b$st.json')); r=d['roofline']; b=d['config']['ssts_per_gpu_per_step']
print('streams $st value', d['value'], 'us/SST', round(r['device_ms_per_sst']*1000,2), {k: round(v/b*1000,2) for k,v in r['stage_ms_per_step'].items()})"
done
