set -u
cd /root/repo
for cfg in "640 2" "640 1" "320 4" "320 5" "192 8"; do
  set -- $cfg
  SDB_EMIT_THREADS=$1 SDB_EMIT_WG_PER_CU=$2 SDB_LIBRARY=libslatedb_amd_pt.so timeout -k 10 120 python3 scripts/phase_times.py > gpurun_out/pt_$1_$2.log 2>&1 || exit $?
  echo "== $cfg"; grep "k_emit waves\|total  " gpurun_out/pt_$1_$2.log | tail -2
  SDB_EMIT_THREADS=$1 SDB_EMIT_WG_PER_CU=$2 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-verify > gpurun_out/b_$1_$2.log 2>&1 || exit $?
  grep -o '"emit": [0-9.]*' gpurun_out/b_$1_$2.log
done
