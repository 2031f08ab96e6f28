#!/bin/bash
# zlib / zstd chain depth 16 (default) vs 8 vs 4: ratio and time on D1 and JSON values
set -o pipefail
mkdir -p gpurun_out/czd
for lib in libslatedb_amd.so libslatedb_amd_czd8.so libslatedb_amd_czd4.so; do
  SDB_CODECS=zlib,zstd SDB_LIBRARY=$lib timeout -k 10 300 python -u scripts/bench_configs.py --compress --reps 3 > gpurun_out/czd/$lib.log 2>&1 || exit 1
  echo "== $lib"; grep '^{' gpurun_out/czd/$lib.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['what'][12:60], d['ms'], d['ratio_device'], d['sample_ratio_library'])"
done
