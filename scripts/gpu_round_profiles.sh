#!/bin/bash
# Refresh every measured number committed under profiles/ in one GPU call (round tag $TAG, default r3):
#   1. bench.py default run (oracle verify + CPU baseline)               -> rp/bench.json
#   2. rocprofv3 --kernel-trace --stats over the bench, one stream        -> rp/enc/
#   3. PMC passes FETCH_SIZE, WRITE_SIZE over the bench                    -> rp/pmc_*/
#   4. scripts/bench_configs.py (every config, CPU baselines)             -> rp/configs.jsonl
#   5. kernel traces: configs[2] decode, configs[3] bloom, compaction, codecs, lookups, the compressors,
#      the single-SST (configs[1]) sequence -> rp/{dec,bloom,compact,codec,lookup,compress,single}/
#   6. PMC FETCH / WRITE of the bloom, the compaction and the decode      -> rp/pmc_{bloom,compact,dec}_*/
#   7. SQ counter passes over the encode and the decode                   -> rp/sq_{enc,dec}/
# Then on the host: python3 scripts/collect_profiles.py $TAG
# Stops at the first failing step.  PART=1: steps 1-4, PART=2: steps 5-7 (two gpurun calls), default both.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/rp
PART=${PART:-all}
[ "$PART" = 2 ] || { rm -rf $O; }
mkdir -p $O
step() {  # name timeout command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 < /dev/null
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
if [ "$PART" != 2 ]; then
step bench 400 python3 bench.py
grep '^{' $O/bench.log > $O/bench.json; cut -c1-300 $O/bench.json
step enc 300 rocprofv3 --kernel-trace --stats -d $O/enc -o run --output-format csv -- python3 bench.py --streams 1 --steps 100 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 0
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 120 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0
done
step configs 600 python3 scripts/bench_configs.py
grep '^{' $O/configs.log > $O/configs.jsonl; cut -c1-200 $O/configs.jsonl
fi
[ "$PART" = 1 ] && { echo done; exit 0; }
step dec 300 rocprofv3 --kernel-trace --stats -d $O/dec -o run --output-format csv -- python3 scripts/bench_configs.py --decode --no-granular --reps 5 --cpu-seconds 0
step bloom 200 rocprofv3 --kernel-trace --stats -d $O/bloom -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 20
step compact 300 rocprofv3 --kernel-trace --stats -d $O/compact -o run --output-format csv -- python3 scripts/bench_configs.py --compact --reps 8
step codec 400 rocprofv3 --kernel-trace --stats -d $O/codec -o run --output-format csv -- python3 scripts/bench_configs.py --codec --reps 3
step lookup 200 rocprofv3 --kernel-trace --stats -d $O/lookup -o run --output-format csv -- python3 scripts/bench_configs.py --lookup --reps 10
step compress 400 rocprofv3 --kernel-trace --stats -d $O/compress -o run --output-format csv -- python3 scripts/bench_configs.py --compress --reps 3
step single 200 rocprofv3 --kernel-trace --stats -d $O/single -o run --output-format csv -- python3 scripts/single_sst.py
for w in bloom:--bloom compact:--compact dec:--decode; do
  n=${w%%:*}; f=${w#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_${n}_$c 120 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_${n}_$c -o run --output-format csv -- python3 scripts/bench_configs.py $f --reps 3 --no-granular --cpu-seconds 0
  done
done
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  step sq_enc_$i 120 rocprofv3 --kernel-trace --pmc $grp -d $O/sq_enc/p$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0
  step sq_dec_$i 120 rocprofv3 --kernel-trace --pmc $grp -d $O/sq_dec/p$i -o run --output-format csv -- python3 scripts/bench_configs.py --decode --no-granular --reps 2 --cpu-seconds 0
done <<EOF2
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
EOF2
python3 scripts/pmc_kernels.py $O/sq_enc/p* > $O/sq_enc_summary.txt && python3 scripts/pmc_kernels.py $O/sq_dec/p* > $O/sq_dec_summary.txt
echo done
