#!/bin/bash
# bloom binning in k_facts, three builds: old (two-pass, one LDS round trip per probe), twopass (probes batched),
# main (one pass into slot-capacity buckets up to 64 KiB of LDS, batched) -- kernel times, VALU, then tests
set -u
export TMPDIR=/tmp
O=gpurun_out/bin2
rm -rf $O; mkdir -p $O
for lib in libslatedb_amd_old.so libslatedb_amd_twopass.so libslatedb_amd.so; do
  SDB_LIBRARY=$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/t_$lib -o run --output-format csv -- python3 bench.py --streams 1 --steps 40 --warmup 5 --no-cpu --no-verify --single-steps 100 --stage-steps 0 > $O/t_$lib.log 2>&1 || { echo "trace rc=$?"; exit 1; }
  echo "== $lib"; grep -E 'k_facts|k_seg|k_emit<' $O/t_$lib/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
  SDB_LIBRARY=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d $O/p_$lib -o run --output-format csv -- python3 bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/p_$lib.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
  python3 scripts/pmc_kernels.py $O/p_$lib | grep -E 'k_facts' | cut -c1-300
done
for lib in libslatedb_amd_twopass.so libslatedb_amd.so; do
SDB_LIBRARY=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_prefix.py tests/test_gpu_block_sizes.py > $O/tests_$lib.log 2>&1; rc=$?; tail -1 $O/tests_$lib.log; [ $rc -eq 0 ] || exit $rc
done
