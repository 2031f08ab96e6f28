#!/bin/bash
# k_emit grid per builder with two builders: 112 / 128 (default) / 144 / 160 workgroups
set -o pipefail
mkdir -p gpurun_out/egrid
for i in 1 2; do
for g in 112 128 144 160; do
  SDB_EMIT_GRID=$g timeout -k 10 200 python3 bench.py --streams 2 --steps 600 --no-cpu --no-verify --stage-steps 0 --single-steps 0 > gpurun_out/egrid/g$g.$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/egrid/g$g.$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$g', d['value'], d['concurrent_builders'])"
done
done
