#!/bin/bash
# Round-2 GPU check: parity tests (-m gpu) then a short bench.  Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_gputests.log 2>&1
rc=$?
tail -5 gpurun_out/r2_gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 --no-cpu > gpurun_out/r2_bench_quick.json 2> gpurun_out/r2_bench_quick.err
rc=$?
cat gpurun_out/r2_bench_quick.json; tail -3 gpurun_out/r2_bench_quick.err
exit $rc
