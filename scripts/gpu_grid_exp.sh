set -u
# streams grid batch (grid 0: the builders hint's default)
for cfg in "2 0 8" "3 128 8" "4 128 8" "2 144 8" "2 0 4" "2 0 16"; do
  set -- $cfg
  S=$1; G=$2; B=$3
  if [ "$G" = 0 ]; then unset SDB_EMIT_GRID; else export SDB_EMIT_GRID=$G; fi
  timeout -k 10 200 python3 bench.py --steps 24 --warmup 6 --no-cpu --no-verify --streams $S --batch $B --single-steps 0 > gpurun_out/g_${S}_${G}_${B}.log 2>&1 || { echo "fail $S $G $B"; tail -5 gpurun_out/g_${S}_${G}_${B}.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/g_${S}_${G}_${B}.log') if l.startswith('{')][0])
print('streams $S grid $G batch $B value', d['value'], 'ms/step', d['ms_per_step'])"
done
