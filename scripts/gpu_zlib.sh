#!/bin/bash
# zlib iteration: the codec tests (incl. decode-once), then the zlib codec bench line and its kernel stats
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/zl
rm -rf $O; mkdir -p $O
step() {  # name timeout command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 < /dev/null
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/$n.log; exit $rc; }
}
step tests 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_codec_once.py tests/test_gpu_codec_write.py -x -q --timeout 200 --timeout-method thread
tail -1 $O/tests.log
SDB_CODECS=${SDB_CODECS:-zlib} step codec 300 python3 scripts/bench_configs.py --codec --reps 3
grep "^{" $O/codec.log | cut -c1-420; grep -o '"device_compressed_once": {[^}]*}' $O/codec.log || true
SDB_CODECS=${SDB_CODECS:-zlib} step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/bench_configs.py --codec --reps 3
grep -E "k_zl|k_ent" $O/prof/run_kernel_stats.csv | cut -c1-160
for v in ${ZL_VARIANTS:-}; do  # variant libraries (make variant NAME=v) on the same bench line
  SDB_LIBRARY=libslatedb_amd_$v.so SDB_CODECS=zlib step codec_$v 300 python3 scripts/bench_configs.py --codec --reps 3
  echo "[$v]"; grep -o '"once_ms": [0-9.]*\|"device_compressed_once": {[^}]*}' $O/codec_$v.log || true
done
echo done
