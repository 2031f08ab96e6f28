#!/bin/bash
# k_seg candidate walks over four-block jump tables: phase marks (timing build), kernel times, encode tests
set -u
export TMPDIR=/tmp
O=gpurun_out/seg
rm -rf $O; mkdir -p $O
SDB_LIBRARY=libslatedb_amd_pt.so timeout -k 10 200 python3 scripts/phase_times.py > $O/phase.log 2>&1 || { echo "phase rc=$?"; exit 1; }
head -8 $O/phase.log
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --streams 1 --steps 40 --warmup 5 --no-cpu --no-verify --single-steps 100 --stage-steps 0 > $O/t.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python3 - <<'PY'
import csv,glob,statistics as st
f=glob.glob('gpurun_out/seg/t/*kernel_trace.csv')[0]
d={}
for r in csv.DictReader(open(f)):
    n=r['Kernel_Name']
    for k in ('k_facts','k_seg','k_anchor','k_blocks','k_emit<','k_emit_big'):
        if k in n: d.setdefault((k,int(r['Grid_Size_Y'])),[]).append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
print(' | '.join('%s y%d %.1f'%(k,y,st.median(v)) for (k,y),v in sorted(d.items())))
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_block_sizes.py tests/test_gpu_compaction.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; exit $rc
