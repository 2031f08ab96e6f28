#!/bin/bash
# Measurement session: phase timing build, secondary configs, HBM traffic PMC passes of the bench.
# Stops at the first crash/timeout.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
if [ -z "${SKIP_PT:-}" ]; then
  SDB_LIBRARY=libslatedb_amd_pt.so timeout -k 10 180 python3 scripts/phase_times.py > gpurun_out/phase.log 2>&1
  rc=$?; echo "phase rc=$rc"; cat gpurun_out/phase.log | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${SKIP_CONFIGS:-}" ]; then
  timeout -k 10 400 python3 scripts/bench_configs.py ${CONFIG_ARGS:-} > gpurun_out/configs.log 2>&1
  rc=$?; echo "configs rc=$rc"; grep -v amdgpu.ids gpurun_out/configs.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${SKIP_PMC:-}" ]; then
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/$grp -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/pmc/$grp.log 2>&1
    rc=$?; echo "pmc $grp rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
