#!/bin/bash
# k_facts cost split: kernel times and SQ counters of the main build, the SipHash-less and the binning-less
# diagnostic builds, and --bpk 0; then the decode tests at the new default (descending emit order)
set -u
export TMPDIR=/tmp
O=gpurun_out/facts
rm -rf $O; mkdir -p $O
B="python3 bench.py --streams 1 --steps 40 --warmup 5 --no-cpu --no-verify --single-steps 0 --stage-steps 0"
run() {  # name lib extra-args
  local n=$1 lib=$2; shift 2
  SDB_LIBRARY=$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- $B "$@" > $O/$n.log 2>&1 || { echo "$n trace rc=$?"; exit 1; }
  SDB_LIBRARY=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d $O/p_$n -o run --output-format csv -- python3 bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0 "$@" > $O/p_$n.log 2>&1 || { echo "$n pmc rc=$?"; exit 1; }
  echo "== $n"; python3 scripts/pmc_kernels.py $O/p_$n | grep -E 'k_facts|k_seg' | cut -c1-400
  grep -E 'k_facts|k_seg|k_emit<' $O/$n/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
}
run base libslatedb_amd.so
run nohash libslatedb_amd_nohash.so
run nobin libslatedb_amd_nobin.so
run bpk0 libslatedb_amd.so --bpk 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_failfast.py tests/test_descending.py tests/test_gpu_parity.py tests/test_gpu_block_sizes.py tests/test_gpu_compaction.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; exit $rc
