#!/bin/bash
# batched bloom binning in k_facts: kernel times + VALU, the encode / bloom parity tests, a short headline bench
set -u
export TMPDIR=/tmp
O=gpurun_out/bin
rm -rf $O; mkdir -p $O
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --streams 1 --steps 40 --warmup 5 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/t.log 2>&1 || { echo "trace rc=$?"; exit 1; }
grep -E 'k_facts|k_seg|k_emit<' $O/t/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d $O/p -o run --output-format csv -- python3 bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/p.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
python3 scripts/pmc_kernels.py $O/p | grep -E 'k_facts' | cut -c1-400
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_prefix.py tests/test_gpu_block_sizes.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 1000 --cpu-seconds 2 > $O/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' $O/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['one_stream'], d['single_sst'], d.get('concurrent_builders'))"
