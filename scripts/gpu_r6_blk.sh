#!/bin/bash
# k_blocks chain walk over four-block jumps vs the previous build: tests first, then
# the headline bench (one builder, two, single SST) on both builds
set -u
export TMPDIR=/tmp
O=gpurun_out/blk
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_block_sizes.py tests/test_gpu_compaction.py tests/test_gpu_prefix.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for lib in libslatedb_amd_prev.so libslatedb_amd.so; do
  SDB_LIBRARY=$lib timeout -k 10 200 python3 bench.py --steps 400 --no-cpu --no-verify --stage-steps 0 > $O/b_$lib.$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  grep '^{' $O/b_$lib.$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['one_stream']['device_ms_per_sst'], d['single_sst']['device_ms_per_sst'], d['concurrent_builders'])"
done
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --streams 1 --steps 40 --warmup 5 --no-cpu --no-verify --single-steps 100 --stage-steps 0 > $O/t.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python3 - <<'PY'
import csv,glob,statistics as st
f=glob.glob('gpurun_out/blk/t/*kernel_trace.csv')[0]
d={}
for r in csv.DictReader(open(f)):
    n=r['Kernel_Name']
    for k in ('k_facts','k_seg','k_anchor','k_blocks','k_emit<','k_emit_big'):
        if k in n: d.setdefault((k,int(r['Grid_Size_Y'])),[]).append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
print(' | '.join('%s y%d %.1f'%(k,y,st.median(v)) for (k,y),v in sorted(d.items())))
PY
