set -o pipefail
export SDB_SETS=d1
SDB_CODECS=zlib,zstd SDB_LIBRARY=libslatedb_amd_czd1.so timeout -k 10 200 python -u scripts/bench_configs.py --compress --reps 3 > gpurun_out/cz_var_d1.log 2>&1 &&
SDB_CODECS=zstd SDB_LIBRARY=libslatedb_amd_czne.so timeout -k 10 200 python -u scripts/bench_configs.py --compress --reps 3 > gpurun_out/cz_var_ne.log 2>&1
