// sdb_encode.h — kernel arguments and LDS geometry of the SST encoder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slatedb_amd.h"

namespace sdb {

constexpr uint32_t kChunk = 2048;            // entries per chunk (K3 / K5)
constexpr uint32_t kResolveLds = 96 * 1024;  // LDS budget of the resolve tables (u16 exits)
// k_emit's CRC tables: slicing-by-8 tables + x^256 byte tables + 6 combine-tree steps (36 KiB), or
// (SDB_EMIT_CRC_MFMA) the matrix-core CRC's weights + the tree steps (sdb_crc_mfma.h, 56 KiB): 43.1 vs
// 41.0 us per SST (r5) — the emit's LDS is not its bound, and 32 dependent MFMAs per block add latency
#ifndef SDB_EMIT_CRC_MFMA
#define SDB_EMIT_CRC_SLICE
#endif
#ifdef SDB_EMIT_CRC_SLICE
constexpr uint32_t kCrcLds = 36 * 1024;
#else
constexpr uint32_t kCrcLds = 56 * 1024;
#endif
constexpr uint32_t kImgCap = 4096 + 64;      // LDS block image per wave (fast path)
constexpr uint32_t kStageCap = 4096;         // value staging per wave (LDS-DMA, 1 KiB per instruction), in place
constexpr uint32_t kStageGuard = 64;         // LDS bytes before each image the value stage may use
constexpr uint32_t kKeyStageCap = 1024;      // key staging per wave
// k_emit's piece path (blocks over one image): a row it can stage with other rows' pieces
constexpr uint32_t kPieceRowMax = 4000, kPieceKeyMax = 960, kPieceValMax = 3968;
constexpr uint32_t kSegLook = 1024;           // k_seg: max lookahead entries staged past the chunk
constexpr uint32_t kSegSpan = kChunk + kSegLook;
constexpr uint32_t kSegThreads = 512;          // four workgroups per CU (kSegLds)
constexpr uint32_t kFactsThreads = 1024;      // k_facts: a chunk (= a fused bloom tile) per workgroup
constexpr uint32_t kFactsPerT = 2;            //   entries per thread
constexpr uint32_t kFactsEntries = kFactsThreads * kFactsPerT;
constexpr uint32_t kSegLds = (2 * kSegSpan + 4) * 4 + kChunk * 6;  // 36 KiB: four workgroups per CU
constexpr uint32_t kSegLdsMax = 64 * 1024;          // k_seg's LDS with the fused bloom binning
constexpr uint32_t kHashPerT = kChunk / kSegThreads;  // chunk entries (hashes) per k_seg thread
#ifndef SDB_EMIT_WAVES
#define SDB_EMIT_WAVES 16
#endif
// SDB_EMIT_WAVES waves per workgroup, 1 per CU: each wave assembles one block while the next one's data
// is in flight (16 waves: 128 VGPRs each, which hold it without spilling)
constexpr uint32_t kEmitThreads = 64 * SDB_EMIT_WAVES;
constexpr uint32_t kEmitWgPerCu = 1;
constexpr uint32_t kEmitWaveLds = kStageGuard + kImgCap + 16 + kKeyStageCap + 64 * 16;  // guard, image, key stage, spans
constexpr uint32_t kEmitLds = kCrcLds + 16 + (kEmitThreads / 64) * kEmitWaveLds;  // tables, ticket, waves
constexpr uint32_t kEnumLds = kChunk * 16 + 11 * kChunk * 2;  // block list + 11 lifting levels (nb <= kChunk = 2^11)
constexpr uint32_t kEnumTabLds = 11 * kChunk * 2;  // k_enum's table walk (aliases the lifting levels)
constexpr uint32_t kGroupThreads = 1024;
constexpr uint32_t kEnumThreads = 512;         // two workgroups per CU (76 KiB LDS, 85 VGPRs)
constexpr uint32_t kGroupLds = kResolveLds;         // group tables, or the single-workgroup resolve

// bloom build plan (sdb_bloom.hip): 2^sb-bit slices, T-key binning tiles
struct BloomPlan {
    uint32_t k, m;        // probes per key, bitmap bits
    uint32_t sb;          // log2 bits per slice
    uint32_t nslices, T, tiles;
    uint32_t one_pass;    // bin straight into per-slice LDS buckets of cap u16 (bloom_bin_core)
    uint32_t pad;
    uint64_t mmod;        // Lemire fastmod constant: floor((2^64 - 1) / m) + 1
};
struct BloomSlots {
    uint32_t *count;  // tiles x nslices: run length of each (tile, slice) slot (kSlotOverflow: too long)
    uint32_t *slot;   // (nslices x tiles) x cap probes, slice-major: u16 offsets in the slice when
                      // sb <= 16 (half the traffic), else u32 bit positions
    uint32_t cap;
};

struct BlockDesc {  // one per block, written by k_enum, streamed by k_emit (56 bytes)
    uint32_t s, e;        // entries [s, e)
    uint64_t off;         // byte offset of the block in the data section
    uint64_t vs, ve, ks, ke;  // value / key byte ranges of the block
    uint32_t bb, pad;     // encoded bytes incl. CRC
};

struct EncodeArgs {
    // batch (device)
    const uint8_t *key_bytes;
    const uint64_t *key_off;
    const uint8_t *val_bytes;
    const uint64_t *val_off;
    const uint8_t *kind;
    const uint64_t *seq;
    const int64_t *create_ts;
    const int64_t *expire_ts;
    const uint8_t *ts_mask;
    uint64_t n;
    // params
    uint32_t block_size;
    uint32_t restart_interval;
    uint32_t version;
    uint32_t wal;           // WAL SST: no compute_index_key (no prefix panic), index_key_len 0
    uint32_t nchunks;
    uint32_t seg_look;      // lookahead entries staged by k_seg (covers the longest possible block)
    // workspace
    uint32_t *lcp;
    uint32_t *szr, *sznr;   // per entry (k_facts): restart-row size, non-restart size (V1: both the row size)
    uint64_t *hd;           // per entry (k_facts, fused bloom): h0 | d0 << 32, first probe and step
    uint32_t nfacts;        // k_facts workgroups (partials: stat_part / err_part are per facts workgroup)
    uint32_t *row_scratch;  // per entry: row offsets of slow-path blocks
    uint32_t *next;
    uint32_t *bbytes;
    uint32_t *tab_exit;
    uint32_t *tab_cnt;
    uint64_t *tab_bytes;
    uint32_t *anchor_e;     // nchunks+1
    uint32_t *anchor_blk;   // nchunks+1
    uint64_t *anchor_byte;  // nchunks+1
    unsigned long long *err;
    uint32_t *wmax;
    uint32_t *slow_count;
    uint32_t *slow_list;
    uint32_t *big_count;    // blocks over one k_emit image whose rows fit pieces (k_emit_big)
    uint32_t *big_list;
    BlockDesc *desc;
    uint64_t *stat_part;    // per k_facts workgroup: raw key, raw val, puts, deletes, merges
    uint32_t *huge_part;    // per k_facts workgroup (= chunk): 1 if a row is too large for k_emit's piece path
    uint32_t *wmax_part;    // per chunk: longest candidate block (entries)
    unsigned long long *err_part;  // per k_facts workgroup: min (entry << 8 | code) of the checks (~0: none)
    uint32_t *gtab_exit;    // per group of kGroup chunks, seg_look candidates: composed transfer table
    uint32_t *gtab_cnt;
    uint64_t *gtab_bytes;
    uint32_t *mode;         // k_group -> k_enum: 1 = compose the tables, 0 = anchors were walked
    uint32_t group;         // chunks per group (host: ~sqrt(nchunks))
    // bloom fused into the encode: k_seg hashes and bins each chunk (tile = chunk), k_enum fills
    uint32_t bloom_fused;
    BloomPlan bpl;
    BloomSlots bq;
    uint8_t *bloom_out;
    uint32_t *done;         // [0] k_emit workgroups finished (the last one writes the summary); [1] block ticket
    uint32_t nprep_wg;
    uint32_t seg_lds;       // k_seg's dynamic LDS bytes
    // outputs (device)
    uint8_t *out_data;
    uint64_t *out_block_off;
    uint32_t *out_block_first;
    uint32_t *out_index_key_len;
    uint16_t *out_block_stats;
    uint64_t data_cap, block_cap;
    sdb_sst_summary *summary;
    uint64_t bloom_len;
    uint32_t num_probes, filter_built;
    const uint64_t *bloom_len_dev;  // prefix-extractor filter: the device-counted length (~0: error)
};

// Workspace layout for n entries (all offsets 256-byte aligned).  Everything up to `bloom_rep` depends
// only on n (and whether a filter is built), so the kernels recompute the layout on the device from
// the SST's workspace base; the bloom slots come last and are sized on the host.
struct EncodeWorkspace {
    uint64_t lcp, szr, sznr, hd, row_scratch, next, bbytes, tab_exit, tab_cnt, tab_bytes;
    uint64_t anchor_e, anchor_blk, anchor_byte, err, wmax, slow_count, slow_list, big_count, big_list, desc, stat_part,
        huge_part, wmax_part,
        bloom_rep;
    uint64_t err_part, done, gtab_exit, gtab_cnt, gtab_bytes, mode, blen;
    uint64_t total;
};
uint64_t bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes);
uint64_t encode_bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes);
__host__ __device__ inline EncodeWorkspace encode_workspace_offsets(uint64_t n, bool has_filter) {
    EncodeWorkspace w{};
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint64_t r = off;
        off += (bytes + 255) & ~255ull;
        return r;
    };
    uint64_t nc = (n + kChunk - 1) / kChunk;
    w.lcp = take(4 * (n + 1));
    w.szr = take(4 * (n + 1));
    w.sznr = take(4 * (n + 1));
    w.hd = take(0);  // (the fused bloom bins inside k_facts: no per-entry hash array)
    (void)has_filter;
    w.row_scratch = take(4 * (n + 1));
    w.next = take(4 * (n + 1));
    w.bbytes = take(4 * (n + 1));
    w.tab_exit = take(4 * (nc * kSegLook + 1));   // per chunk: seg_look candidate entry points
    w.tab_cnt = take(4 * (nc * kSegLook + 1));
    w.tab_bytes = take(8 * (nc * kSegLook + 1));
    w.anchor_e = take(4 * (nc + 2));
    w.anchor_blk = take(4 * (nc + 2));
    w.anchor_byte = take(8 * (nc + 2));
    w.err = take(8);
    w.wmax = take(4);
    w.slow_count = take(4);
    w.slow_list = take(4 * (n + 1));
    w.big_count = take(4);
    w.big_list = take(4 * (n + 1));
    w.desc = take(sizeof(BlockDesc) * (n + 1));
    const uint64_t nf = (n + kFactsEntries - 1) / kFactsEntries;
    w.stat_part = take(8 * 5 * (nf + 1));
    w.huge_part = take(4 * (nf + 1));
    w.wmax_part = take(4 * (nc + 1));
    w.err_part = take(8 * (nf + 1));
    w.done = take(8);
    w.gtab_exit = take(4 * (nc * kSegLook + 1));  // one table per group (<= one per chunk)
    w.gtab_cnt = take(4 * (nc * kSegLook + 1));
    w.gtab_bytes = take(8 * (nc * kSegLook + 1));
    w.mode = take(4);
    w.blen = take(8);   // prefix-extractor filters: the filter length the device counted
    w.bloom_rep = off;  // bloom slots or the prefix filter's scratch (host-sized) last
    w.total = off;
    return w;
}
inline EncodeWorkspace encode_workspace_layout(uint64_t n, uint64_t filter_bytes, uint32_t num_probes) {
    EncodeWorkspace w = encode_workspace_offsets(n, filter_bytes != 0);
    w.total = w.bloom_rep + ((filter_bytes ? encode_bloom_workspace_bytes(n, num_probes, filter_bytes) : 0) + 255) / 256 * 256;
    return w;
}
uint64_t prefix_workspace_bytes(uint64_t n);
hipError_t launch_bloom_prefix(const uint8_t *key_bytes, const uint64_t *key_off, const int32_t *lens, uint64_t n,
                               uint32_t bpk, uint32_t kind, uint32_t arg, uint32_t whole, uint8_t *bitmap, uint64_t cap,
                               uint64_t *bloom_len, void *ws, hipStream_t st);
hipError_t launch_bloom_match(const uint8_t *bitmap, uint64_t bytes, uint32_t k, uint32_t whole, uint32_t kind,
                              uint32_t arg, const uint8_t *key_bytes, const uint64_t *key_off, const uint8_t *is_prefix,
                              const int32_t *qlens, uint64_t n, uint8_t *result, hipStream_t st);

// ------------------------------------------------------------------------------------------------
// A launch set: up to kMaxSsts independent SSTs with the same SsTableFormat knobs encoded by ONE
// launch sequence (blockIdx.y = SST for the per-SST grids; k_emit spreads every SST's blocks over one
// persistent grid).  The compaction / flush callers run several builders at once (l0_flush_parallelism,
// subcompactions: config.rs:1081, 1383-1390); batching them fills the GPU with the latency-bound
// segmentation kernels of all of them at once.  Passed by value (kernel arguments).
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kMaxSsts = 8;
enum WsField {
    kWsLcp = 0, kWsSzr, kWsSznr, kWsHd, kWsRowScratch, kWsNext, kWsBbytes, kWsTabExit, kWsTabCnt, kWsTabBytes,
    kWsAnchorE, kWsAnchorBlk, kWsAnchorByte, kWsErr, kWsWmax, kWsSlowCount, kWsSlowList, kWsBigCount, kWsBigList,
    kWsDesc, kWsStatPart, kWsHugePart, kWsWmaxPart, kWsBloomRep, kWsErrPart, kWsDone, kWsGtabExit, kWsGtabCnt,
    kWsGtabBytes, kWsMode, kWsBlen, kWsFields
};
struct SstSlot {
    const uint8_t *key_bytes;
    const uint64_t *key_off;
    const uint8_t *val_bytes;
    const uint64_t *val_off;
    const uint8_t *kind;
    const uint64_t *seq;
    const int64_t *create_ts;
    const int64_t *expire_ts;
    const uint8_t *ts_mask;
    uint64_t n;
    uint8_t *out_data;
    uint64_t *out_block_off;
    uint32_t *out_block_first;
    uint32_t *out_index_key_len;
    uint16_t *out_block_stats;
    uint64_t data_cap, block_cap;
    sdb_sst_summary *summary;
    uint8_t *bloom_out;
    uint64_t bloom_len;
    uint8_t *ws;              // this SST's workspace (256-byte aligned)
    uint32_t num_probes, filter_built, bloom_fused, has_filter_ws;  // has_filter_ws: hd in the layout
    uint32_t nchunks, nfacts, group, slot_cap;
    uint32_t prefix_bloom, pad2;  // the filter is a prefix-extractor one: its length is device-counted
    BloomPlan bpl;            // fused bloom plan (bloom_fused)
    // encode_workspace_offsets(n, has_filter_ws) in 256-byte units, filled on the host (fill_ws_layout):
    // the kernels load them instead of re-deriving the layout's 64-bit offset chain on the scalar unit
    uint32_t wso[kWsFields];
};
struct SstSet {
    uint32_t count;
    uint32_t block_size, restart_interval, version, wal, seg_look;
    uint32_t max_facts, max_chunks, max_groups, max_tiles, max_slices, pad;
    SstSlot s[kMaxSsts];
};

// EncodeArgs of SST i of a set (workspace carved from the slot's base; host and device).
__host__ __device__ inline EncodeArgs make_args(const SstSet &P, uint32_t i) {
    const SstSlot &s = P.s[i];
    EncodeArgs a{};
    a.key_bytes = s.key_bytes;
    a.key_off = s.key_off;
    a.val_bytes = s.val_bytes;
    a.val_off = s.val_off;
    a.kind = s.kind;
    a.seq = s.seq;
    a.create_ts = s.create_ts;
    a.expire_ts = s.expire_ts;
    a.ts_mask = s.ts_mask;
    a.n = s.n;
    a.block_size = P.block_size;
    a.restart_interval = P.restart_interval;
    a.version = P.version;
    a.wal = P.wal;
    a.nchunks = s.nchunks;
    a.seg_look = P.seg_look;
    uint8_t *b = s.ws;
    auto W = [&](int f) { return b + ((uint64_t)s.wso[f] << 8); };
    a.lcp = (uint32_t *)W(kWsLcp);
    a.szr = (uint32_t *)W(kWsSzr);
    a.sznr = (uint32_t *)W(kWsSznr);
    a.hd = (uint64_t *)W(kWsHd);
    a.nfacts = s.nfacts;
    a.row_scratch = (uint32_t *)W(kWsRowScratch);
    a.next = (uint32_t *)W(kWsNext);
    a.bbytes = (uint32_t *)W(kWsBbytes);
    a.tab_exit = (uint32_t *)W(kWsTabExit);
    a.tab_cnt = (uint32_t *)W(kWsTabCnt);
    a.tab_bytes = (uint64_t *)W(kWsTabBytes);
    a.anchor_e = (uint32_t *)W(kWsAnchorE);
    a.anchor_blk = (uint32_t *)W(kWsAnchorBlk);
    a.anchor_byte = (uint64_t *)W(kWsAnchorByte);
    a.err = (unsigned long long *)W(kWsErr);
    a.wmax = (uint32_t *)W(kWsWmax);
    a.slow_count = (uint32_t *)W(kWsSlowCount);
    a.slow_list = (uint32_t *)W(kWsSlowList);
    a.big_count = (uint32_t *)W(kWsBigCount);
    a.big_list = (uint32_t *)W(kWsBigList);
    a.desc = (BlockDesc *)W(kWsDesc);
    a.stat_part = (uint64_t *)W(kWsStatPart);
    a.huge_part = (uint32_t *)W(kWsHugePart);
    a.wmax_part = (uint32_t *)W(kWsWmaxPart);
    a.err_part = (unsigned long long *)W(kWsErrPart);
    a.gtab_exit = (uint32_t *)W(kWsGtabExit);
    a.gtab_cnt = (uint32_t *)W(kWsGtabCnt);
    a.gtab_bytes = (uint64_t *)W(kWsGtabBytes);
    a.mode = (uint32_t *)W(kWsMode);
    a.group = s.group;
    a.bloom_fused = s.bloom_fused;
    a.bpl = s.bpl;
    {  // bloom slots (BloomSlots, sdb_bloom.hip): counts then slots, 256-byte aligned
        uint8_t *q = W(kWsBloomRep);
        a.bq.count = (uint32_t *)q;
        a.bq.slot = (uint32_t *)(q + (((uint64_t)s.bpl.tiles * s.bpl.nslices * 4 + 255) & ~255ull));
        a.bq.cap = s.slot_cap;
    }
    a.bloom_out = s.bloom_out;
    a.done = (uint32_t *)W(kWsDone);
    a.nprep_wg = s.nchunks;
    a.seg_lds = kSegLds;
    a.out_data = s.out_data;
    a.out_block_off = s.out_block_off;
    a.out_block_first = s.out_block_first;
    a.out_index_key_len = s.out_index_key_len;
    a.out_block_stats = s.out_block_stats;
    a.data_cap = s.data_cap;
    a.block_cap = s.block_cap;
    a.summary = s.summary;
    a.bloom_len = s.bloom_len;
    a.num_probes = s.num_probes;
    a.filter_built = s.filter_built;
    a.bloom_len_dev = s.prefix_bloom ? (uint64_t *)W(kWsBlen) : nullptr;
    return a;
}

// The slot's workspace layout (wso) from its n and has_filter_ws (host, after both are set).
inline void fill_ws_layout(SstSlot &s) {
    const EncodeWorkspace w = encode_workspace_offsets(s.n, s.has_filter_ws != 0);
    const uint64_t off[kWsFields] = {w.lcp, w.szr, w.sznr, w.hd, w.row_scratch, w.next, w.bbytes, w.tab_exit, w.tab_cnt,
                                     w.tab_bytes, w.anchor_e, w.anchor_blk, w.anchor_byte, w.err, w.wmax, w.slow_count,
                                     w.slow_list, w.big_count, w.big_list, w.desc, w.stat_part, w.huge_part, w.wmax_part,
                                     w.bloom_rep, w.err_part, w.done, w.gtab_exit, w.gtab_cnt, w.gtab_bytes, w.mode, w.blen};
    for (int f = 0; f < kWsFields; f++) s.wso[f] = (uint32_t)(off[f] >> 8);
}

// Enqueue the encode of every SST of the set on `st` (one launch sequence).
hipError_t launch_encode_set(const SstSet &P, size_t bin_lds, size_t fill_lds, hipStream_t st);
hipError_t launch_encode_empty(EncodeArgs a, hipStream_t st);
hipError_t launch_encode_prep(const SstSet &P, hipStream_t st);  // k_facts, k_seg, k_group only

// stage timing (diagnostics)
enum Stage { kStBloom = 0, kStFacts, kStSeg, kStAnchor, kStBlocks, kStEmit, kStEmitBig, kStBloomFill, kNumStages };
void stage_mark(hipStream_t st, int stage, bool begin);
bool stage_timing_on();

// bloom (sdb_bloom.hip)

// tile_keys: keys per binning tile (0: the standalone build's choice; the fused encode bins per chunk)
BloomPlan bloom_plan(uint64_t n, uint32_t k, uint64_t bitmap_bytes, uint32_t tile_keys = 0);
uint64_t bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes);
// ws: bloom_workspace_bytes(...) of scratch, or NULL (device-scope atomics; slow)
hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes, void *ws,
                              hipStream_t st);
hipError_t launch_bloom_query(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes,
                              const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint8_t *result, hipStream_t st);

}  // namespace sdb
static_assert(sdb::kSegSpan % sdb::kSegThreads == 0 && sdb::kChunk % 64 == 0, "k_seg geometry");
static_assert(sdb::kEmitLds <= 160 * 1024, "k_emit LDS");
static_assert(sizeof(sdb::SstSet) <= 4096, "SstSet is passed as kernel arguments");
