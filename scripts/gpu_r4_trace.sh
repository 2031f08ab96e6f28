#!/bin/bash
# Round 4, first call: the driver's bench shape (20 steps, 5 warmup) three times, then one kernel trace
# of the same shape, to see whether the two builders' kernels overlap or queue behind k_emit.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r4t
rm -rf $O; mkdir -p $O
step() {  # name timeout command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 < /dev/null
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for i in 1 2 3 4 5; do
  case $i in 4) export SDB_EMIT_POOL=8;; 5) export SDB_EMIT_POOL=16;; esac
  step drv$i 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS:-}
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/drv$i.log') if l.startswith('{')][0]); r=d['roofline']
print('pool', '${SDB_EMIT_POOL:-0}', 'value', d['value'], 'ms/SST', r['device_ms_per_sst'], 'one', d['one_stream']['device_ms_per_sst'], 'single', d['single_sst']['device_ms_per_sst'])"
done
unset SDB_EMIT_POOL
step trace 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --stage-steps 0 --single-steps 0 ${BENCH_ARGS:-}
echo done
