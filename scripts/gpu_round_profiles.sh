#!/bin/bash
# Refresh every measured number committed under profiles/ in one GPU call:
#   1. bench.py default run (oracle verify + CPU baseline)          -> gpurun_out/rp/bench.json
#   2. rocprofv3 --kernel-trace --stats over the bench, one stream   -> gpurun_out/rp/enc/
#   3. PMC passes FETCH_SIZE, WRITE_SIZE (one counter per pass)      -> gpurun_out/rp/pmc_*/
#   4. scripts/bench_configs.py (configs[2], configs[3], E2E)        -> gpurun_out/rp/configs.jsonl
#   5. rocprofv3 --kernel-trace --stats over the decode of configs[2] -> gpurun_out/rp/dec/
#   6. SQ counter passes over the encode bench and the configs[2] decode -> gpurun_out/rp/sq_{enc,dec}/
# Then on the host: python3 scripts/collect_profiles.py r2
# Stops at the first failing step.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/rp
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log > $O/bench.json; cut -c1-300 $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/enc -o run --output-format csv -- python3 bench.py --streams 1 --steps 100 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/enc.log 2>&1
rc=$?; echo "rocprof enc rc=$rc"
[ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python3 scripts/bench_configs.py > $O/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep '^{' $O/configs.log > $O/configs.jsonl; cut -c1-200 $O/configs.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dec -o run --output-format csv -- python3 scripts/bench_configs.py --decode --no-granular --reps 5 --cpu-seconds 0 > $O/dec.log 2>&1
rc=$?; echo "rocprof dec rc=$rc"
[ $rc -eq 0 ] || exit $rc
G="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
i=0
while read -r grp; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/sq_enc/p$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0 > $O/sq_enc_$i.log 2>&1
  rc=$?; echo "sq enc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/sq_dec/p$i -o run --output-format csv -- python3 scripts/bench_configs.py --decode --no-granular --reps 2 --cpu-seconds 0 > $O/sq_dec_$i.log 2>&1
  rc=$?; echo "sq dec $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<EOF2
$G
EOF2
python3 scripts/pmc_summary.py $O/sq_enc > $O/sq_enc/summary.txt && python3 scripts/pmc_summary.py $O/sq_dec > $O/sq_dec/summary.txt
