#!/bin/bash
# Diagnostic builds of k_emit (wrong output by design): per-stage device times of the batched bench per
# build in $EXPS ("base" = the product library).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for x in ${EXPS:-base}; do
  lib=libslatedb_amd_$x.so; [ "$x" = base ] && lib=libslatedb_amd.so
  SDB_LIBRARY=$lib timeout -k 10 120 python3 bench.py --steps ${STEPS:-200} --warmup 5 --no-cpu --no-verify --single-steps 0 ${BENCH_ARGS:-} > gpurun_out/emit_$x.json 2> gpurun_out/emit_$x.err
  rc=$?; [ $rc -eq 0 ] || { echo "== $x rc=$rc"; tail -3 gpurun_out/emit_$x.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/emit_$x.json')); r=d['roofline']; b=d['config']['ssts_per_gpu_per_step']
print('== $x', 'us/SST', round(r['device_ms_per_sst']*1000,1), {k: round(v/b*1000,1) for k,v in r['stage_ms_per_step'].items()})"
done
