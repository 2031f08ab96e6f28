#!/bin/bash
# PMC passes (one rocprofv3 run per line of $PMC_GROUPS, default: HBM bytes + SQ groups) over $CMD.
#   CMD="python3 scripts/bench_configs.py --bloom --reps 3" OUT=gpurun_out/pmc bash scripts/gpu_pmc_groups.sh
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
rm -rf $OUT; mkdir -p $OUT
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1 < /dev/null
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<PMC_END
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU}
PMC_END
python3 scripts/pmc_kernels.py $OUT/p* > $OUT/summary.txt; cat $OUT/summary.txt
