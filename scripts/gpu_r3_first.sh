#!/bin/bash
# Round-3 first call: GPU suite at HEAD, default bench, then configs[3] bloom kernel trace + FETCH/WRITE/SQ passes.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/bloom -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 20 > $O/bloom.log 2>&1
rc=$?; echo "bloom trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d $O/bpmc_$n -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 3 > $O/bpmc_$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
