#!/bin/bash
# PMC passes over the f3 decompression kernels, one codec at a time (SDB_CODECS): FETCH_SIZE, WRITE_SIZE
# and two SQ groups, each its own rocprofv3 run; summaries per codec -> gpurun_out/pc/<codec>.txt
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/pc
rm -rf $O; mkdir -p $O
for c in ${PMC_CODECS:-lz4 snappy zstd zlib}; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    SDB_CODECS=$c timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $grp -d $O/$c/p$i -o run --output-format csv -- python3 scripts/bench_configs.py --codec --reps 3 > $O/$c.p$i.log 2>&1 || { echo "$c p$i failed"; tail -5 $O/$c.p$i.log; exit 1; }
  done
  python3 scripts/pmc_kernels.py $O/$c/p* > $O/$c.txt
  echo "== $c"; grep -E "k_dz|k_ent|k_zl" $O/$c.txt | cut -c1-400
done
echo done
