#!/bin/bash
# Round 5 iteration: the whole -m gpu suite, then the workloads named in $WORK (space separated):
#   enc     bench.py driver shape (20 steps, 5 warmup) without the CPU leg
#   dec     configs[2] decode (bench_configs.py --decode) + its kernel trace stats
#   bsz     every SstBlockSize: encode and decode per SST
#   encv    encode throughput on D2 and D1-L0 (headline shape)
#   bloom   configs[3] bloom + kernel trace stats
#   compact the compaction job + kernel trace stats
#   codec   the f3 decompression workloads + kernel trace stats
#   encprof kernel trace stats of the one-stream bench
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/it
rm -rf $O; mkdir -p $O
step() {  # name timeout command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 < /dev/null
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/$n.log; exit $rc; }
}
if [ -z "${NOTEST:-}" ]; then
  step tests 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
  tail -2 $O/tests.log
fi
for w0 in ${WORK:-}; do
  w=${w0%%:*}; v=""; unset SDB_LIBRARY SDB_DEC_PHASE
  if [ "$w0" != "$w" ]; then v=${w0#*:}; export SDB_LIBRARY=libslatedb_amd_$v.so; echo "== variant $v"; fi
  [ "$v" = pt ] && export SDB_DEC_PHASE=1
  case $w in
    enc) step enc$v 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu ${v:+--no-verify}
         python3 -c "
import json; d=json.loads([l for l in open('$O/enc$v.log') if l.startswith('{')][0]); r=d['roofline']
print('enc value', d['value'], 'ms/SST', r['device_ms_per_sst'], 'frac', r['frac'], 'single', d['single_sst']['device_ms_per_sst'], {k: round(v/8*1000,1) for k,v in r['stage_ms_per_step'].items()}, 'one', d['one_stream'])" ;;
    encx) step encx 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu ${ENCX_ARGS:-}
         python3 -c "
import json; d=json.loads([l for l in open('$O/encx.log') if l.startswith('{')][0]); r=d['roofline']
print('encx ${ENCX_ARGS:-}: value', d['value'], 'ms/SST', r['device_ms_per_sst'], {k: round(v/8*1000,1) for k,v in r['stage_ms_per_step'].items()})" ;;
    footer) step footer 200 python3 scripts/bench_configs.py --footer
         grep '^{' $O/footer.log | cut -c1-300 ;;
    encprof) step encprof 300 rocprofv3 --kernel-trace --stats -d $O/encprof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu --no-verify --single-steps 0 --stage-steps 0 ;;
    dec) step dec$v 300 python3 scripts/bench_configs.py --decode --no-granular --reps 10 --cpu-seconds 0
         grep '^{\|ticks' $O/dec$v.log | cut -c1-400
         [ -n "$v" ] || step decprof 300 rocprofv3 --kernel-trace --stats -d $O/decprof -o run --output-format csv -- python3 scripts/bench_configs.py --decode --no-granular --reps 5 --cpu-seconds 0 ;;
    bsz) step bsz$v 400 python3 scripts/bench_block_sizes.py
         grep "^{" $O/bsz$v.log | cut -c1-300 ;;
    encv) step encv 300 python3 scripts/bench_configs.py --encode --reps 20
         grep '^{' $O/encv.log | cut -c1-400 ;;
    bloom) step bloom$v 200 python3 scripts/bench_configs.py --bloom --reps 20
         grep '^{' $O/bloom$v.log | cut -c1-300
         [ -n "$v" ] || step bloomprof 200 rocprofv3 --kernel-trace --stats -d $O/bloomprof -o run --output-format csv -- python3 scripts/bench_configs.py --bloom --reps 20 ;;
    compact) step compact 300 python3 scripts/bench_configs.py --compact --reps 8
         grep '^{' $O/compact.log | cut -c1-300
         step compactprof 300 rocprofv3 --kernel-trace --stats -d $O/compactprof -o run --output-format csv -- python3 scripts/bench_configs.py --compact --reps 8 ;;
    codec) [ -z "$v" ] || step codectest$v 300 python3 -u -m pytest tests/test_gpu_codec.py -x -q --timeout 200 --timeout-method thread
         SDB_CODECS=${SDB_CODECS:-lz4,snappy,zlib,zstd} step codec$v 400 python3 scripts/bench_configs.py --codec --reps 3
         grep "^{" $O/codec$v.log | cut -c1-520
         [ -n "$v" ] || step codecprof 400 rocprofv3 --kernel-trace --stats -d $O/codecprof -o run --output-format csv -- python3 scripts/bench_configs.py --codec --reps 3 ;;
  esac
done
for f in $O/*prof/run_kernel_stats.csv; do [ -f $f ] && { echo "== $f"; cut -d, -f1-8 $f | head -14; }; done
echo done
