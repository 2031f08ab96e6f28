#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 200 python3 bench.py --batch 1 --streams 1 --steps 100 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 100 > gpurun_out/b1.log 2>&1 || exit 1
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/b1.log") if l.startswith("{")][0])
r = d["roofline"]
print("batch1 value", d["value"], "ms/SST", r["device_ms_per_sst"], {k: round(v * 1000, 1) for k, v in r["stage_ms_per_step"].items()})
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/b1prof -o run --output-format csv -- python3 bench.py --batch 1 --streams 1 --steps 100 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > gpurun_out/b1prof.log 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/b1prof/run_kernel_stats.csv | head -14
