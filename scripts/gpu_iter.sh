#!/bin/bash
# One iteration on the GPU box: smoke -> gpu tests -> bench -> rocprof kernel stats of the bench.
# Stops at the first failure that is not a plain test failure (crash, abort, timeout).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${SMOKE_T:-240} python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${TEST_T:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-verify > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/prof/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print("%-45s %6s %9.1f us" % (r["Name"][:45], r["Calls"], float(r["AverageNs"]) / 1e3))
    break
PY
exit $rc
