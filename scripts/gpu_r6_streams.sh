#!/bin/bash
# builders per GPU: 2 (default) vs 3 vs 4, same box
set -o pipefail
mkdir -p gpurun_out/streams
for i in 1 2; do
for s in 2 3 4; do
  timeout -k 10 200 python3 bench.py --streams $s --steps 600 --no-cpu --no-verify --stage-steps 0 --single-steps 0 > gpurun_out/streams/s$s.$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/streams/s$s.$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$s', d['value'], d['one_stream']['device_ms_per_sst'], d['concurrent_builders'])"
done
done
