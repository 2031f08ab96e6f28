#!/bin/bash
# k_emit workgroup geometry vs the two-builder pipeline: SDB_EMIT_THREADS x builders (streams).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/geom
mkdir -p $O
for cfg in "1024 2" "768 2" "768 3" "512 2" "512 3" "640 2"; do
  set -- $cfg
  SDB_EMIT_THREADS=$1 timeout -k 10 120 python3 -u bench.py --steps 600 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 0 --streams $2 > $O/b_$1_$2.json 2> $O/b_$1_$2.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 $O/b_$1_$2.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$O/b_$1_$2.json')); r=d['roofline']
print('threads $1 streams $2: value', d['value'], 'us/SST', round(r['device_ms_per_sst']*1000,2), 'frac', r['frac'])"
done
