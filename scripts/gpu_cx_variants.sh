mkdir -p gpurun_out/cxv
for v in "" vd ve; do
  L=libslatedb_amd_$v.so; [ -z "$v" ] && L=libslatedb_amd.so
  
  SDB_LIBRARY=$L timeout -k 10 200 python3 scripts/bench_configs.py --compact --reps 15 > gpurun_out/cxv/b_$v.log 2>&1 || exit 1
  echo "== $L"; grep '^{' gpurun_out/cxv/b_$v.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['ms_wall'], d['bit_exact_vs_oracle'])"
done
