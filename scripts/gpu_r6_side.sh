#!/bin/bash
# k_emit_big on a stream forked beside k_emit (shared completion counter) vs the serial launch: tests first, then
# the headline bench (one builder, two, single SST) on both builds
set -u
export TMPDIR=/tmp
O=gpurun_out/side
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_block_sizes.py tests/test_gpu_compaction.py tests/test_gpu_prefix.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for lib in libslatedb_amd_serial.so libslatedb_amd.so; do
  SDB_LIBRARY=$lib timeout -k 10 200 python3 bench.py --steps 400 --no-cpu --no-verify --stage-steps 0 > $O/b_$lib.$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  grep '^{' $O/b_$lib.$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['one_stream']['device_ms_per_sst'], d['single_sst']['device_ms_per_sst'], d['concurrent_builders'])"
done
done
