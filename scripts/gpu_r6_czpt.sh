#!/bin/bash
# compressor phase ticks (diagnostic build), then the write-side bench line and tests
set -o pipefail
mkdir -p gpurun_out
SDB_LIBRARY=libslatedb_amd_czpt.so timeout -k 10 300 python -u scripts/cz_phases.py > gpurun_out/cz_pt.log 2>&1 &&
bash scripts/gpu_r6_cz.sh
