// sdb_compact.h — kernel arguments of the compaction output side (sdb_compact.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slatedb_amd.h"
#include "sdb_encode.h"

namespace sdb {

constexpr uint32_t kMaxRuns = SDB_MAX_RUNS;
#ifndef SDB_MERGE_TILE
#define SDB_MERGE_TILE 1024
#endif
#ifndef SDB_MERGE_THREADS
#define SDB_MERGE_THREADS 512
#endif
constexpr uint32_t kMergeTile = SDB_MERGE_TILE;  // merged positions per k_mg_tiles / k_mg_emit workgroup
constexpr uint32_t kMergeThreads = SDB_MERGE_THREADS;

struct RunDesc {  // sdb_run + the run's first global entry index
    uint64_t n, base;
    const uint8_t *key_arena;
    const uint64_t *key_off;
    const uint8_t *val_base;
    const uint64_t *val_off;
    const uint32_t *val_len;
    const uint64_t *seq;
    const uint8_t *flags;
    const int64_t *create_ts;
    const int64_t *expire_ts;
};

struct MergeArgs {
    uint32_t nruns, ntiles;
    uint32_t raw, pad;           // raw: no retention, no merge-operand check (every entry kept as it is)
    uint64_t total;
    sdb_retention ret;
    sdb_merged_out out;
    // workspace
    uint64_t *pfx;               // per global entry: key bytes [L0, L0 + 8), big-endian, zero padded
    uint32_t *lcp0;              // L0: the prefix every key of the (sorted) runs shares
    uint64_t *perm;              // merged position -> global entry
    uint8_t *start;              // merged position: first version of its key
    uint8_t *dec;                // merged position: 0 drop, 1 keep, 2 keep as a tombstone
    uint64_t *tile_sum;          // per tile: kept entries, key bytes, value bytes (exclusive offsets after k_mg_scan)
    uint64_t *bound;             // per 256 entries (k_mg_rank workgroup) and side: the first / last entry's count in each run
    unsigned long long *err;     // run order violations: min (global entry << 8 | code)
    unsigned long long *err_merge;  // merge operands (MergeOperatorRequiredIterator): min merged position << 8 | code
    unsigned long long *metric;  // expired values, expired merges
    const unsigned long long *gate;  // NULL, or (entry << 8 | status) of a failed input (~0: none): no merge
    RunDesc r[kMaxRuns];
};
static_assert(sizeof(MergeArgs) < 4000, "MergeArgs is passed as kernel arguments");

struct MergeWorkspace {
    uint64_t pfx, perm, start, dec, tile_sum, bound, err, err_merge, metric, lcp0, total;
};
inline MergeWorkspace merge_workspace_layout(uint64_t total) {
    MergeWorkspace w{};
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint64_t r = off;
        off += (bytes + 255) & ~255ull;
        return r;
    };
    const uint64_t ntiles = (total + kMergeTile - 1) / kMergeTile;
    w.pfx = take(8 * (total + 1));
    w.perm = take(8 * (total + 1));
    w.start = take(total + 1);
    w.dec = take(total + 1);
    w.tile_sum = take(24 * (ntiles + 1));
    w.bound = take(16 * (uint64_t)kMaxRuns * ((total + 255) / 256 + 1));  // k_mg_bounds: 2 x runs per 256 entries
    w.err = take(8);
    w.err_merge = take(8);
    w.metric = take(16);
    w.lcp0 = take(8);
    w.total = off;
    return w;
}

sdb_status build_merge_args(const sdb_run *runs, uint32_t nruns, const sdb_retention *ret, const sdb_merged_out *out,
                            void *workspace, uint64_t workspace_bytes, MergeArgs *a, bool raw = false);
// A merged stream as an sdb_run (the per-entry value lengths and RowFlags the runs carry): val_len[i],
// flags[i] for i < n (device, written on st).
hipError_t launch_merged_as_run(const sdb_merged_out &out, uint64_t n, uint32_t *val_len, uint8_t *flags, hipStream_t st);
// merge + retention (+ emit when `emit`), all on `st`
hipError_t launch_merge(const MergeArgs &a, bool emit, hipStream_t st);
hipError_t launch_merge_emit(const MergeArgs &a, hipStream_t st);

// SST cuts over the chain tables of a prep-only encode set of one slot (launch_encode_prep).  n_real
// (device, or NULL = the slot's n): the stream's true length when the slot covers a padded stream; the
// walk stops there (a block before it is the same in both streams) and cuts past it are not recorded.
hipError_t launch_cuts(const SstSet &P, uint64_t max_sst_size, uint64_t *cut, uint64_t cap, uint64_t *num,
                       hipStream_t st, const uint64_t *n_real = nullptr);

// ---- sdb_compactor_run_ssts (decode inside the job) ----
struct CxInputs {  // kernel arguments: the input SSTs' blocks, in input order (tables in device memory)
    uint32_t n, nruns;
    uint64_t base;                     // the decoder's arena: block k = base + start[k] (mod 2^64)
    uint64_t nblocks;                  // blocks of every input
    const uint8_t *const *data;        // n: each input's data section
    const uint64_t *const *block_off;  // n: each input's BlockMeta offsets
    const uint64_t *first_block;       // n + 1: prefix of num_blocks
    const uint64_t *run_block;         // nruns + 1: first block of each run, then the total
    const uint64_t *run_entry;         // nruns + 1: declared first entry of each run, then the total
    uint64_t key_bytes;                // declared total key bytes
};
// block k of the job -> arena offsets [start, end)
hipError_t launch_cx_blocks(const CxInputs &in, uint64_t *start, uint64_t *end, hipStream_t st);
// the decode's summary and run boundaries against the declared counts -> *gate (~0: the merge may run)
hipError_t launch_cx_gate(const CxInputs &in, const sdb_decode_summary *dsum, const unsigned long long *dec_err,
                          const uint64_t *block_entry_start, unsigned long long *gate, hipStream_t st);
// sdb_sst_cuts over a padded stream whose true length is *n_real (device)
sdb_status sst_cuts_padded(const sdb_kv_batch *batch, const sdb_sst_params *params, uint64_t max_sst_size,
                           uint64_t *cut_start, uint64_t cut_cap, uint64_t *num_ssts, void *workspace,
                           uint64_t workspace_bytes, hipStream_t stream, const uint64_t *n_real);
// merged positions [summary.num_out + 1, cap]: empty entries (offsets = the totals), so a prep over the
// padded stream reads defined bytes
hipError_t launch_merge_pad(const sdb_merged_out &out, uint64_t cap, hipStream_t st);

// out[2i], out[2i+1] = key_off[cut[i]], val_off[cut[i]] for i <= ns
hipError_t launch_cut_offsets(const uint64_t *cut, const uint64_t *num, const uint64_t *key_off, const uint64_t *val_off,
                              uint64_t *out, hipStream_t st);

}  // namespace sdb
