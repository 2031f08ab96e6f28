#!/bin/bash
# One GPU session: smoke -> gpu tests -> short bench.  Stops at the first crash/timeout
# (exit codes other than 0/1), so a faulting kernel is never re-run in the same call.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${SMOKE_T:-300} python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${TEST_T:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 ${BENCH_T:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-seconds 5} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
