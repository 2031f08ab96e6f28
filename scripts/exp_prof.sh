#!/bin/bash
# rocprofv3 kernel stats of `$EXP_CMD` for each experiment library in $LIBS
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/expprof
export TMPDIR=/tmp
i=0
for lib in $LIBS; do
  i=$((i+1))
  SDB_LIBRARY=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/expprof/e$i -o run --output-format csv -- python3 $EXP_CMD > gpurun_out/expprof/e$i.log 2>&1
  rc=$?; echo "== $lib rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/expprof/e$i/run_kernel_stats.csv')):
    if r['Name'].startswith('sdb::'): print('   %-40s %8.1f us' % (r['Name'][:40], float(r['AverageNs'])/1e3))
"
done
