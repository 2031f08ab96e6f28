#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over a short bench (or $PMC_CMD); per-kernel averages -> gpurun_out/pmc_sq/summary.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_sq
export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_sq/p$i -o run --output-format csv -- ${PMC_CMD:-python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --single-steps 0 --stage-steps 0} > gpurun_out/pmc_sq/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU}
GROUPS
python3 scripts/pmc_summary.py gpurun_out/pmc_sq > gpurun_out/pmc_sq/summary.txt
cat gpurun_out/pmc_sq/summary.txt
