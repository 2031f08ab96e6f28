#!/bin/bash
# compressor at chain depth 8: write-side tests, the compress bench lines and their kernel trace
set -u
export TMPDIR=/tmp
O=gpurun_out/czf
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_codec_write.py tests/test_footer.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 scripts/bench_configs.py --compress --reps 3 > $O/compress.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' $O/compress.log > $O/compress.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 scripts/bench_configs.py --compress --reps 3 > $O/t.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
