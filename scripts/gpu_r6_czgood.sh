#!/bin/bash
# zlib / zstd good length 16 (default) vs 8, nice length 128 vs 64: ratio and time on D1 and JSON values
set -o pipefail
mkdir -p gpurun_out/czgn
for lib in libslatedb_amd.so libslatedb_amd_czg8.so libslatedb_amd_czn64.so; do
  SDB_CODECS=zlib,zstd SDB_LIBRARY=$lib timeout -k 10 300 python -u scripts/bench_configs.py --compress --reps 3 > gpurun_out/czgn/$lib.log 2>&1 || exit 1
  echo "== $lib"; grep '^{' gpurun_out/czgn/$lib.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['what'][12:60], d['ms'], d['ratio_device'], d['sample_ratio_library'])"
done
