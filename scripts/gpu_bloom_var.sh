#!/bin/bash
# configs[3] bloom with alternative libraries ($LIBS), one bench line each (bit-exact checked).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/bvar
for L in libslatedb_amd.so $LIBS; do
  SDB_LIBRARY=$L timeout -k 10 200 python3 scripts/bench_configs.py --bloom --reps 20 > gpurun_out/bvar/$L.log 2>&1 || exit 1
  echo "$L $(grep '^{' gpurun_out/bvar/$L.log | cut -c1-150)"
done
