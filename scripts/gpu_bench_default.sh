#!/bin/bash
# The driver's bench command (defaults), then a one-line digest of its JSON.
set -u
cd "$(dirname "$0")/.."
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_default.log; exit $rc; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_default.log") if l.startswith("{")][0])
r = d["roofline"]
print("value", d["value"], "ms_step", d["ms_per_step"], "single", d["single_sst"]["device_ms_per_sst"],
      "one_stream", d["one_stream"], "copy", r["measured_copy_GBps"], "k_emit", r["k_emit"], "cpu", d["cpu_baseline"]["value"])
PY
