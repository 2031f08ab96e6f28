#!/bin/bash
# Encode pipeline stage times per SST (HIP events, one stream) for bench.py argument sets in $ARGSETS
# (separated by ';'), no CPU leg, no oracle verify.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/encexp
i=0
IFS=';' read -ra SETS <<< "${ARGSETS:-}"
for a in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 python3 -u bench.py --steps 400 --warmup 10 --no-cpu --no-verify --single-steps 0 $a > gpurun_out/encexp/b$i.json 2> gpurun_out/encexp/b$i.err < /dev/null
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/encexp/b$i.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/encexp/b$i.json')); r=d['roofline']; b=d['config']['ssts_per_gpu_per_step']
print('[$a]', 'value', d['value'], 'us/SST', round(r['device_ms_per_sst']*1000,2), 'one_stream', round(d['one_stream']['device_ms_per_sst']*1000,2) if d['one_stream'] else None, {k: round(v/b*1000,2) for k,v in r['stage_ms_per_step'].items()})"
done
