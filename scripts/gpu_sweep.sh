#!/bin/bash
# bench variants over env tuning knobs: each line of $SWEEP is "ENV=.. ENV=.." (empty = default).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
i=0
while read -r envs; do
  i=$((i+1))
  env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu ${BENCH_EXTRA:-} > gpurun_out/sweep/s$i.log 2>&1
  rc=$?
  echo "[$envs] rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sweep/s$i.log | head -1) $(grep -o '"stage_ms": {[^}]*}' gpurun_out/sweep/s$i.log)"
  [ $rc -eq 0 ] || exit $rc
done <<LINES
${SWEEP:-}
LINES
