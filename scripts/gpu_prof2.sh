#!/bin/bash
# kernel stats of the bench and of the secondary configs (rocprofv3 --kernel-trace --stats)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "${CONFIGS:-}" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o run --output-format csv -- python3 scripts/bench_configs.py $CONFIGS > gpurun_out/prof_cfg.log 2>&1
rc=$?; echo "rocprof configs rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
python3 - <<'PY'
import csv
for d in ["gpurun_out/prof", "gpurun_out/prof_cfg"]:
    try:
        rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
    except FileNotFoundError:
        continue
    print("==", d)
    for r in rows:
        print("%-60s %6s %10.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
