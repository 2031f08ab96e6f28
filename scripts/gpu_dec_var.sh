#!/bin/bash
# configs[2] decode (ascending / descending) and decode at every block size for the library variants
# $LIBS (default library first), bit-exactness checked by the benches.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/decvar
mkdir -p $O
for L in libslatedb_amd.so $LIBS; do
  SDB_LIBRARY=$L timeout -k 10 300 python3 scripts/bench_configs.py --decode --no-granular --reps 10 --cpu-seconds 0 > $O/$L.dec.log 2>&1 || exit 1
  SDB_LIBRARY=$L SDB_BLOCK_SIZES=4096,8192,16384,65536 timeout -k 10 300 python3 scripts/bench_block_sizes.py > $O/$L.bs.log 2>&1 || exit 1
  echo "== $L"; grep '^{' $O/$L.dec.log | cut -c1-110; grep '^{' $O/$L.bs.log | python3 -c "
import json,sys
print([(d['block_size'], d['decode_us_per_sst'], d['decode_keys_ok']) for d in map(json.loads, sys.stdin)])"
done
