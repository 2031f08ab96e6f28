// sdb_encode.hip — SST data-section encoder for gfx950.
//
// Replaces EncodedSsTableBuilder::{add, finish_block, build} (slatedb/src/sst_builder.rs:224-417)
// with BlockBuilderV2/V1 (format/block_v2.rs:118-240, format/block.rs:76-218), the row codecs
// (format/row_codec_v2.rs:127-169, format/row.rs:159-198) and the per-block CRC32 of
// compress_and_transform (format/sst.rs:525-554).
//
// The greedy block fill of the reference (BlockBuilderV2::would_fit, block_v2.rs:151-164) is a
// sequential chain b -> next(b).  It is parallelised as:
//   K1 prep     one thread per entry: LCP vs previous key, restart/non-restart row sizes, checks,
//               stats.
//   K2 next     one thread per entry b: next(b) = end of a block that would start at b, and its
//               encoded size.
//   K3 chunk    one workgroup per chunk of kChunk entries: pointer jumping in LDS gives, for every
//               entry point e of the chunk, the first block start past the chunk plus the blocks
//               and bytes on the way (a chunk transfer table).
//   K4 resolve  one workgroup: the chunk tables are composed by a Blelloch up-sweep in LDS and the
//               single chain from entry 0 is pushed down the tree (O(log K) depth) -> per-chunk
//               anchors (first block start, block index, byte offset).
//   K5 emit     one workgroup per chunk: binary lifting enumerates the chunk's block starts, then
//               one wave per block stages the block's keys/values in LDS with 16-byte loads,
//               assembles the rows, restart table and count in an LDS image, computes the CRC32
//               (slicing-by-8 per lane + GF(2) shift-combine across the wave) and writes the block
//               with 16-byte stores.
//   K6 slow     blocks larger than the LDS image (oversized first entries, huge block sizes) are
//               assembled directly in HBM by one workgroup each.
#include <stdlib.h>

#include <atomic>
#include <mutex>

#include "sdb_bloom.h"
#include "sdb_crc.h"
#include "sdb_crc_mfma.h"

namespace sdb {

// Phase timestamps (diagnostic builds with -DSDB_PHASE_TIMING): per workgroup of the instrumented
// kernel, s_memtime at each phase mark of thread 0 -> g_phase[blockIdx][mark].  A mark adds its own
// barrier in timing builds only: it never stands in for a barrier the algorithm needs.
#ifndef SDB_SEG_WAVES
#define SDB_SEG_WAVES 8
#endif
#ifdef SDB_PHASE_TIMING
__device__ uint64_t g_phase[1024][8];
#define PHASE_MARK(i)                                                              \
    do {                                                                           \
        __syncthreads();                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 1024) g_phase[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
__device__ uint64_t g_wave_phase[8192][8];
__device__ uint64_t g_phase_enum[1024][8];
#define PHASE_MARK_E(i)                                                                  \
    do {                                                                                 \
        __syncthreads();                                                                 \
        if (threadIdx.x == 0 && blockIdx.x < 1024) g_phase_enum[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
__device__ uint64_t g_wave_rt[8192][4];  // k_emit per wave: s_memrealtime start/end, s_memtime start/end
#define WAVE_T(var)                                     \
    uint64_t var = __builtin_amdgcn_s_memtime();        \
    __builtin_amdgcn_s_waitcnt(0xC07F) /* lgkmcnt(0) */
#define PHASE_MARK_AT(slot, i)                                                        \
    do {                                                                          \
        __syncthreads();                                                          \
        if (threadIdx.x == 0) g_phase[slot][i] = __builtin_amdgcn_s_memtime();   \
    } while (0)
#else
#define PHASE_MARK(i) \
    do {              \
    } while (0)
#define PHASE_MARK_AT(slot, i) \
    do {                       \
    } while (0)
#define PHASE_MARK_E(i) \
    do {                \
    } while (0)
#define WAVE_T(var) \
    do {            \
    } while (0)
#endif


// ------------------------------------------------------------------------------------------------
// Per-entry facts: LCP vs the previous key, restart / non-restart row sizes, reference errors.
// ------------------------------------------------------------------------------------------------
struct EntryFacts {
    uint32_t lcp, s_r, s_nr;
    uint64_t klen, vlen;
    uint8_t kind;
    int err;
};

// The facts are computed in three steps so a thread can issue the loads of several entries before
// it waits: offsets/flags, then the first 16 bytes of this and the previous key, then the rest.
struct FactsIn {
    uint64_t pko, ko0, ko1, vo0, vo1;
    uint64_t pk0, pk1, ck0, ck1;  // first 16 bytes of the previous / this key (masked by length later)
    uint8_t kd, m;
};

SDB_DEV void facts_load_offsets(const EncodeArgs &a, uint64_t i, FactsIn &in) {
    in.ko0 = a.key_off[i];
    in.ko1 = a.key_off[i + 1];
    in.pko = i > 0 ? a.key_off[i - 1] : in.ko0;
    in.vo0 = a.val_off[i];
    in.vo1 = a.val_off[i + 1];
    in.kd = a.kind ? a.kind[i] : 0;
    in.m = a.ts_mask ? a.ts_mask[i] : 0;
}

SDB_DEV void facts_load_keys(const EncodeArgs &a, FactsIn &in) {
    const uint64_t klen = in.ko1 - in.ko0, plen = in.ko0 - in.pko;
    uint64_t n = klen < plen ? klen : plen;
    n = n < 16 ? n : 16;
    in.pk0 = in.ck0 = in.pk1 = in.ck1 = 0;
    if (n) {
        const uint32_t n0 = (uint32_t)(n < 8 ? n : 8);
        in.pk0 = load8(a.key_bytes + in.pko, n0);
        in.ck0 = load8(a.key_bytes + in.ko0, n0);
        if (n > 8) {
            in.pk1 = load8(a.key_bytes + in.pko + 8, (uint32_t)(n - 8));
            in.ck1 = load8(a.key_bytes + in.ko0 + 8, (uint32_t)(n - 8));
        }
    }
}

SDB_DEV EntryFacts facts_finish(const EncodeArgs &a, uint64_t i, const FactsIn &in) {
    EntryFacts f;
    const uint64_t klen = in.ko1 - in.ko0;
    const uint8_t kd = in.kd, m = in.m;
    const uint64_t vlen = (kd == SDB_KIND_TOMBSTONE) ? 0 : (in.vo1 - in.vo0);
    uint32_t lcp = 0;
    int err = 0;
    if (kd > SDB_KIND_TOMBSTONE) err = SDB_INVALID_ARGUMENT;
    if (!err && i > 0) {
        const uint64_t plen = in.ko0 - in.pko;
        const uint64_t mn = plen < klen ? plen : klen;
        const uint32_t nmin = (uint32_t)(mn > 0xFFFFFFFFull ? 0xFFFFFFFFull : mn);
        // compute_prefix (block_v2.rs:52-75) on the preloaded 16 bytes, then on from HBM
        const uint32_t n0 = nmin < 8 ? nmin : 8, n1 = nmin < 16 ? nmin - n0 : 8;
        uint64_t x0 = in.pk0 ^ in.ck0, x1 = in.pk1 ^ in.ck1;
        if (n0 < 8) x0 &= (1ull << (8 * n0)) - 1;
        if (n1 < 8) x1 &= (1ull << (8 * n1)) - 1;
        if (x0) lcp = __builtin_ctzll(x0) >> 3;
        else if (x1) lcp = 8 + (__builtin_ctzll(x1) >> 3);
        else if (nmin <= 16) lcp = nmin;
        else lcp = 16 + lcp_bytes(a.key_bytes + in.pko + 16, nmin - 16, a.key_bytes + in.ko0 + 16, nmin - 16);
        // compute_index_key runs on every entry (sst_builder.rs:228): assert on empty keys and
        // out-of-bounds panic when this key is a proper prefix of the previous one (utils.rs:210-216)
        if (klen == 0) err = SDB_EMPTY_KEY;
        else if (!a.wal && plen > 0 && lcp == klen && klen < plen) err = SDB_INVALID_ARGUMENT;
    }
    if (!err && klen == 0) err = SDB_EMPTY_KEY;  // BlockBuilder*::add (block_v2.rs:168-170)
    const uint32_t ts8 = 8u * (((m & SDB_TS_CREATE) != 0) + ((m & SDB_TS_EXPIRE) != 0));
    if (a.version == 2) {
        if (!err && (klen > 0xFFFFFFFFull || vlen > 0xFFFFFFFFull)) err = SDB_LIMIT_EXCEEDED;
        uint32_t kl = (uint32_t)klen, vl = (uint32_t)vlen, suf = kl - lcp;
        // SstRowEntryV2::encoded_size (row_codec_v2.rs:92-116)
        f.s_nr = varint_len(lcp) + varint_len(suf) + varint_len(vl) + suf + vl + 9 + ts8;
        f.s_r = 1 + varint_len(kl) + varint_len(vl) + kl + vl + 9 + ts8;
    } else {
        // SstRowEntry::new asserts (row.rs:73-85)
        if (!err && (klen > 0xFFFF || vlen > 0xFFFFFFFFull)) err = SDB_LIMIT_EXCEEDED;
        // RowEntry::encoded_size with key_prefix_len = 0 (types.rs:64-83)
        f.s_r = (uint32_t)(4 + klen + 9 + ts8 + (kd == SDB_KIND_TOMBSTONE ? 0 : 4 + vlen));
        f.s_nr = f.s_r;
    }
    f.lcp = lcp;
    f.klen = klen;
    f.vlen = vlen;
    f.kind = kd;
    f.err = err;
    return f;
}

SDB_DEV EntryFacts entry_facts(const EncodeArgs &a, uint64_t i) {
    FactsIn in;
    facts_load_offsets(a, i, in);
    facts_load_keys(a, in);
    return facts_finish(a, i, in);
}

// ------------------------------------------------------------------------------------------------
// K0 facts: one thread per entry (a lean, high-occupancy pass, so the loads of many entries are in
// flight per CU): LCP vs the previous key, restart / non-restart row sizes, reference errors, SstStats
// partials per workgroup and, for the fused bloom, filter_hash (filter.rs:196-204) reduced to the
// first probe and step.  Lanes hold consecutive entries: the next entry's offsets and the previous
// key's first 16 bytes come from the neighbour lane by DPP (lane 63 / lane 0 load their own).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kFactsThreads, 8) void k_facts(SstSet P) {
    const EncodeArgs a = make_args(P, blockIdx.y);
    if (blockIdx.x >= a.nfacts) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t blds[];  // fused bloom binning
    __shared__ uint64_t s_part[kFactsThreads / 64][5];
    __shared__ unsigned long long s_err[kFactsThreads / 64];
    __shared__ uint32_t s_huge[kFactsThreads / 64];
    const uint32_t tid = threadIdx.x, lane = (uint32_t)lane_id();
    const uint64_t e0 = (uint64_t)blockIdx.x * kFactsEntries + tid;  // entries e0 + r * kFactsThreads
    const uint64_t n = a.n;
    // all loads of both rounds first (offsets, then the first 16 key bytes), so they overlap
    FactsIn in[kFactsPerT];
#pragma unroll
    for (uint32_t r = 0; r < kFactsPerT; r++) {
        const uint64_t e = e0 + r * kFactsThreads;
        FactsIn &f = in[r];
        f.ko0 = f.ko1 = f.vo0 = f.vo1 = f.pko = 0;
        f.kd = f.m = 0;
        if (e <= n) {
            f.ko0 = a.key_off[e];
            f.vo0 = a.val_off[e];
            if (e < n) {
                f.kd = a.kind ? a.kind[e] : 0;
                f.m = a.ts_mask ? a.ts_mask[e] : 0;
                if (lane == 63) {
                    f.ko1 = a.key_off[e + 1];
                    f.vo1 = a.val_off[e + 1];
                }
                if (lane == 0 && e > 0) f.pko = a.key_off[e - 1];
            }
        }
    }
    // the first 16 bytes of every key (and lane 0's previous key): one unconditional 16-byte load per
    // entry, all in flight together (a load under a branch would make the compiler wait for every
    // earlier one at the join).  A window that would run past the key bytes (a short key at the end
    // of the batch) reads 16 in-bounds bytes of key_off instead and is re-read byte-exactly below.
    const uint64_t ktot = a.key_off[n];
#pragma unroll
    for (uint32_t r = 0; r < kFactsPerT; r++) {
        FactsIn &f = in[r];
        const uint64_t nk = wave_next_lane(f.ko0), nv = wave_next_lane(f.vo0);
        if (lane != 63) {
            f.ko1 = nk;
            f.vo1 = nv;
        }
        const uint64_t e = e0 + r * kFactsThreads;
        const bool live = e < n;
        const uint8_t *safe = (const uint8_t *)a.key_off;  // >= 16 bytes (n + 1 >= 2 offsets)
        const uint8_t *cs = live && f.ko0 + 16 <= ktot ? a.key_bytes + f.ko0 : safe;
        uint4 cw;
        __builtin_memcpy(&cw, cs, 16);
        f.ck0 = (uint64_t)cw.x | (uint64_t)cw.y << 32;
        f.ck1 = (uint64_t)cw.z | (uint64_t)cw.w << 32;
        f.pk0 = f.pk1 = 0;
    }
    // lane 0's previous keys last: their branch joins after every other load is already in flight
#pragma unroll
    for (uint32_t r = 0; r < kFactsPerT; r++) {
        FactsIn &f = in[r];
        const uint64_t e = e0 + r * kFactsThreads;
        if (lane == 0 && e > 0 && e < n && f.pko + 16 <= ktot) {
            uint4 pw;
            __builtin_memcpy(&pw, a.key_bytes + f.pko, 16);
            f.pk0 = (uint64_t)pw.x | (uint64_t)pw.y << 32;
            f.pk1 = (uint64_t)pw.z | (uint64_t)pw.w << 32;
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < kFactsPerT; r++) {  // short keys at the very end of the batch
        FactsIn &f = in[r];
        const uint64_t e = e0 + r * kFactsThreads;
        if (e < n && f.ko0 + 16 > ktot) {
            const uint64_t kl = f.ko1 - f.ko0;
            const uint32_t kn = (uint32_t)(kl < 16 ? kl : 16);
            f.ck0 = f.ck1 = 0;
            if (kn) f.ck0 = load8(a.key_bytes + f.ko0, kn < 8 ? kn : 8);
            if (kn > 8) f.ck1 = load8(a.key_bytes + f.ko0 + 8, kn - 8);
        }
        if (lane == 0 && e > 0 && e < n && f.pko + 16 > ktot) {
            const uint64_t pl = f.ko0 - f.pko;
            const uint32_t pn = (uint32_t)(pl < 16 ? pl : 16);
            f.pk0 = f.pk1 = 0;
            if (pn) f.pk0 = load8(a.key_bytes + f.pko, pn < 8 ? pn : 8);
            if (pn > 8) f.pk1 = load8(a.key_bytes + f.pko + 8, pn - 8);
        }
    }
    uint64_t rk = 0, rv = 0, c = 0;
    uint64_t err = ~0ull;
    bool huge = false;  // a row k_emit's piece path cannot stage (the block goes to the workgroup path)
    uint32_t hh[kFactsPerT], dd[kFactsPerT];
#pragma unroll
    for (uint32_t r = 0; r < kFactsPerT; r++) {
        FactsIn &f = in[r];
        const uint64_t e = e0 + r * kFactsThreads;
        {
            const uint64_t pko = wave_prev_lane(f.ko0), pk0 = wave_prev_lane(f.ck0), pk1 = wave_prev_lane(f.ck1);
            if (lane != 0) {
                f.pko = pko;
                f.pk0 = pk0;
                f.pk1 = pk1;
            } else if (e == 0) {
                f.pko = f.ko0;
            }
        }
        hh[r] = dd[r] = 0;
        if (e < n) {
            const EntryFacts x = facts_finish(a, e, f);
            a.lcp[e] = x.lcp;
            a.szr[e] = x.s_r;
            a.sznr[e] = x.s_nr;
            if (a.bloom_fused) {  // filter_hash (filter.rs:196-204) -> first probe and step
                const uint64_t kl = f.ko1 - f.ko0;
#ifdef SDB_EXP_FACTS_NOHASH  // diagnostic: wrong filter bits by design (cost of SipHash)
                const uint64_t h = (f.ck0 * 0x9E3779B97F4A7C15ull) ^ (f.ck1 + kl);
#else
                const uint64_t h = kl == 16 ? siphash13_16(f.ck0, f.ck1) : siphash13(a.key_bytes + f.ko0, kl);
#endif
                hh[r] = fastmod_u32((uint32_t)h, a.bpl.mmod, a.bpl.m);
                dd[r] = fastmod_u32((uint32_t)(h >> 32), a.bpl.mmod, a.bpl.m);
            }
            if (x.err) {
                const uint64_t ev = (e << 8) | (uint64_t)x.err;
                err = ev < err ? ev : err;
            }
            huge |= x.s_r > kPieceRowMax || x.klen > kPieceKeyMax || x.vlen > kPieceValMax;
            rk += x.klen;
            rv += x.vlen;
            c += (uint64_t)(x.kind == SDB_KIND_VALUE) | ((uint64_t)(x.kind == SDB_KIND_TOMBSTONE) << 20) |
                 ((uint64_t)(x.kind == SDB_KIND_MERGE) << 40);
        }
    }
    // SstStats (sst_builder.rs:225-226, 315-317) and the first error: per-workgroup partials
    rk = wave_sum(rk);
    rv = wave_sum(rv);
    c = wave_sum(c);
    err = wave_readlane(wave_incl_scan_op(err, [](uint64_t x, uint64_t y) { return x < y ? x : y; }), 63);
    const uint32_t w = tid >> 6;
    if (lane == 0) {
        s_part[w][0] = rk;
        s_part[w][1] = rv;
        s_part[w][2] = c & 0xFFFFF;
        s_part[w][3] = (c >> 20) & 0xFFFFF;
        s_part[w][4] = (c >> 40) & 0xFFFFF;
        s_err[w] = err;
    }
    const bool wh = __ballot(huge) != 0;
    if (lane == 0) s_huge[w] = wh ? 1u : 0u;
    __syncthreads();
    if (tid < 5) {
        uint64_t t = 0;
        for (uint32_t q = 0; q < kFactsThreads / 64; q++) t += s_part[q][tid];
        a.stat_part[5 * (uint64_t)blockIdx.x + tid] = t;
    }
    if (tid == 0) {
        unsigned long long m = ~0ull;
        for (uint32_t q = 0; q < kFactsThreads / 64; q++) m = s_err[q] < m ? s_err[q] : m;
        a.err_part[blockIdx.x] = m;  // every workgroup writes its slot: no initialisation needed
        uint32_t h = 0;
        for (uint32_t q = 0; q < kFactsThreads / 64; q++) h |= s_huge[q];
        a.huge_part[blockIdx.x] = h;
    }
    // the fused bloom: this workgroup's kChunk keys are one binning tile (sdb_bloom.h)
    if (a.bloom_fused) {
        const uint64_t k0 = (uint64_t)blockIdx.x * kFactsEntries;
        const uint32_t nk = (uint32_t)((k0 + kFactsEntries < n ? k0 + kFactsEntries : n) - k0);
#ifdef SDB_EXP_FACTS_NOBIN  // diagnostic: every (tile, slice) run empty
        bloom_bin_core<kFactsPerT>(blockIdx.x, hh, dd, 0, a.bpl, a.bq, blds);
#else
        bloom_bin_core<kFactsPerT>(blockIdx.x, hh, dd, nk, a.bpl, a.bq, blds);
#endif
    }
}

// ------------------------------------------------------------------------------------------------
// K1 seg: one workgroup per chunk of kChunk entries, plus a lookahead of seg_look entries (the
// longest block a chunk entry can start) staged in LDS.
//   a. entry facts for the staged span: LCP, errors and stats of the chunk's own entries; row sizes
//      clamped to block_size + 16 (a clamped entry never fits after another one, exactly like the
//      real one) -> LDS;
//   b. V2: P = exclusive prefix of the non-restart sizes, R = prefix of the restart surcharges along
//      each residue class mod restart_interval.  size(b, e) of a block [b, e) is then O(1):
//        2 + P[e] - P[b] + R[last restart] - R[b - ri];
//   c. next(b) = the largest e with size(b, e) <= block_size (at least b + 1): a search started at
//      the estimate block_size / (mean row size) that steps by the size formula (BlockBuilderV2::
//      would_fit, block_v2.rs:151-164: adding an entry keeps the block within block_size);
//      V1 (prefixes against the block's first key) keeps the entry-by-entry walk;
//   d. chains from the seg_look candidate entry points at the chunk start, walked in LDS to the first
//      block start past the chunk: exit, blocks and bytes per candidate (the chunk transfer table).
// ------------------------------------------------------------------------------------------------
SDB_DEV uint32_t walk_size_v2(const EncodeArgs &a, uint64_t j, bool rs) {
    EntryFacts f = entry_facts(a, j);
    return rs ? f.s_r : f.s_nr;
}

SDB_DEV void seg_chunk(const EncodeArgs &a, uint8_t *smem, uint32_t k) {
    uint32_t *s_P = (uint32_t *)smem;          // kSegSpan + 4: prefix of clamped non-restart sizes
    uint32_t *s_R = s_P + kSegSpan + 4;        // kSegSpan: restart surcharge of each entry
    uint32_t *s_bb = s_R + kSegSpan;           // kChunk: encoded block bytes for blocks starting here
    uint16_t *s_nx = (uint16_t *)(s_bb + kChunk);  // kChunk: next(b) - cs (0xFFFF: out of range)
    __shared__ uint32_t s_len[kSegThreads / 64];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t cs = (uint64_t)k * kChunk;
    const uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
    const uint64_t se = ce + a.seg_look < a.n ? ce + a.seg_look : a.n;
    const uint32_t cn = (uint32_t)(ce - cs), sn = (uint32_t)(se - cs);
    const uint64_t bs = a.block_size;
    const uint32_t clampv = (uint32_t)(bs + 16);
    // prefix sums of clamped sizes stay < 2^32 for block sizes up to 1 MiB; beyond that (and for V1)
    // next() walks entry by entry
    const bool v2 = a.version == 2 && bs <= (1u << 20);
    const uint32_t ri = a.restart_interval;
    PHASE_MARK(0);
    // a. row sizes of the staged span (k_facts)
    constexpr uint32_t kPerT = kSegSpan / kSegThreads;
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t zr[kPerT], znr[kPerT];
#pragma unroll
    for (uint32_t u = 0; u < kPerT; u++) {
        const uint32_t x = tid + u * nt;
        zr[u] = znr[u] = 0;
        if (x < sn) {
            zr[u] = a.szr[cs + x];
            znr[u] = a.sznr[cs + x];
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < kPerT; u++) {
        const uint32_t x = tid + u * nt;
        if (x >= sn) continue;
        if (v2) {
            const uint32_t cr = zr[u] < clampv ? zr[u] : clampv, cnr = znr[u] < clampv ? znr[u] : clampv;
            s_P[x] = cnr;
            s_R[x] = cr + 2 - cnr;  // restart row: restart size + its 2-byte offset, instead of cnr
        }
    }
    __syncthreads();
    PHASE_MARK(1);
    // b. P = exclusive prefix of the clamped non-restart sizes (V2): one block scan of the three
    //    strided rows (entry x = tid + u * nt); the restart surcharges stay per entry (s_R)
    if (v2) {
        __shared__ uint32_t s_wt[kPerT * (kSegThreads / 64) + 1];
        const uint32_t wv = tid >> 6;
        uint32_t v[kPerT], inc[kPerT];
#pragma unroll
        for (uint32_t u = 0; u < kPerT; u++) {
            const uint32_t x = tid + u * nt;
            v[u] = x < sn ? s_P[x] : 0;
            inc[u] = wave_incl_scan(v[u]);
            if (lane == 63) s_wt[u * (nt >> 6) + wv] = inc[u];
        }
        __syncthreads();
        if (tid < 64) {
            const uint32_t nw = kPerT * (nt >> 6);
            const uint32_t t = tid < nw ? s_wt[tid] : 0, it = wave_incl_scan(t);
            __builtin_amdgcn_wave_barrier();
            if (tid < nw) s_wt[tid] = it - t;
            if (tid == 63) s_P[sn] = it;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < kPerT; u++) {
            const uint32_t x = tid + u * nt;
            if (x < sn) s_P[x] = s_wt[u * (nt >> 6) + wv] + inc[u] - v[u];
        }
        PHASE_MARK(2);
    }
    __syncthreads();
    PHASE_MARK(3);
    // c. next(b)
    uint32_t maxlen = 0;
    for (uint32_t x = tid; x < cn; x += nt) {
        const uint64_t b = cs + x;
        uint64_t j;        // next(b)
        uint64_t bytes;    // Block::size of [b, j) (+ CRC below)
        if (v2) {
            // size(b, e) for b < e <= sn (clamped sizes; exact whenever it is <= block_size)
            const uint32_t Pb = s_P[x];
            auto size_of = [&](uint32_t e) -> uint64_t {  // + the surcharges of the restart rows x, x + ri, ...
                uint64_t sz = 2ull + (s_P[e] - Pb);
                for (uint32_t r = x; r < e; r += ri) sz += s_R[r];
                return sz;
            };
            // start from an estimate and step (sizes are positive, so size(b, e) grows with e)
            uint32_t lo = x + 1;  // size(b, lo) may exceed block_size: a one-entry block
            uint32_t e = lo;
            {
                const uint32_t w = (x + 64 < sn ? x + 64 : sn) - x;
                const uint32_t mean = (s_P[x + w] - Pb) / w + 1;
                uint32_t est = x + (uint32_t)(bs / mean);
                e = est < lo ? lo : (est > sn ? sn : est);
            }
            if (size_of(e) <= bs) {
                while (e < sn && size_of(e + 1) <= bs) e++;
            } else {
                while (e > lo && size_of(e) > bs) e--;
            }
            j = cs + e;
            if (e == lo) bytes = 2ull + a.szr[b] + 2;  // single row: its true size (unclamped, from HBM)
            else bytes = size_of(e);
            if (e == sn && se < a.n) {
                // the block may continue past the staged span (only for blocks longer than
                // seg_look, i.e. never when seg_look bounds the longest block): walk on from HBM
                uint64_t acc = bytes;
                uint32_t p = e - x, ph = p % ri;
                while (j < a.n) {
                    const bool rs = ph == 0;
                    const uint64_t add = (uint64_t)walk_size_v2(a, j, rs) + (rs ? 2 : 0);
                    if (acc + add > bs) break;
                    acc += add;
                    j++;
                    if (++ph == ri) ph = 0;
                }
                bytes = acc;
            }
        } else if (a.version == 2) {  // huge blocks: V2 walk with sizes from HBM
            uint64_t acc = 2;
            j = b;
            uint32_t p = 0, ph = 0;
            while (j < a.n) {
                const bool rs = ph == 0;
                const uint64_t add = (uint64_t)walk_size_v2(a, j, rs) + (rs ? 2 : 0);
                if (p > 0 && acc + add > bs) break;
                acc += add;
                j++;
                p++;
                if (++ph == ri) ph = 0;
            }
            bytes = acc;
        } else {
            uint64_t acc = 2;
            j = b;
            uint32_t p = 0;
            const uint64_t fko = a.key_off[b];
            const uint32_t fkl = (uint32_t)(a.key_off[b + 1] - fko);
            while (j < a.n) {
                uint32_t prefix = 0;
                if (p > 0) {
                    uint64_t ko = a.key_off[j];
                    prefix = lcp_bytes(a.key_bytes + fko, fkl, a.key_bytes + ko, (uint32_t)(a.key_off[j + 1] - ko));
                }
                uint64_t sr = a.szr[j];
                uint64_t sz = sr - prefix;
                if (p > 0 && acc + sz > bs) break;  // the new entry's 2-byte offset is not counted (block.rs:117-123)
                acc += sz + 2;
                j++;
                p++;
            }
            bytes = acc;
        }
        const uint32_t bb = (uint32_t)(bytes + 4);  // + CRC32 (format/sst.rs:541-552)
        a.next[b] = (uint32_t)j;
        a.bbytes[b] = bb;
        s_bb[x] = bb;
        const uint64_t rel = j - cs;
        s_nx[x] = (uint16_t)(rel < 0xFFFF ? rel : 0xFFFF);
        const uint32_t len = (uint32_t)(j - b);
        maxlen = len > maxlen ? len : maxlen;
    }
    maxlen = wave_max(maxlen);
    if (lane_id() == 0) s_len[tid >> 6] = maxlen;
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0;
        for (uint32_t q = 0; q < nt / 64; q++) m = s_len[q] > m ? s_len[q] : m;
        a.wmax_part[k] = m;
    }
    PHASE_MARK(4);
    // d. chains from the candidate entry points [cs, cs + Wc).  A block that starts before cs and
    //    reaches past cs + x holds the non-restart rows [cs, cs + x], so (V2, clamped sizes <= true
    //    sizes) sum(s_nr[cs .. cs + x]) <= block_size - 2: entry points lie in [cs, cs + x_max + 1].
    __shared__ uint32_t s_wc;
    if (tid == 0) {
        uint32_t wc = a.seg_look;
        if (v2) {
            uint32_t lo = 0, hi = sn;  // largest x in [0, sn] with P[x] - P[0] <= bs - 2
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if ((uint64_t)(s_P[mid] - s_P[0]) + 2 <= bs) lo = mid;
                else hi = mid - 1;
            }
            wc = lo + 1 < wc ? lo + 1 : wc;
        }
        s_wc = wc;
    }
    __syncthreads();
    const uint32_t Wc = s_wc;
    // four-block jumps along the chain (two doubling rounds over the chunk, in the P / R words, which are done
    // with): each candidate's walk below takes a quarter of the dependent LDS steps (~58 -> ~15 per D1 chunk)
    uint32_t *j_nx = s_P;                  // kChunk: exit after up to four blocks (rel, 0xFFFF far) | blocks << 16
    uint64_t *j_bb = (uint64_t *)(s_P + kChunk);  // kChunk: their bytes (8-byte aligned: kChunk is even)
    static_assert(3 * kChunk <= 2 * kSegSpan + 4, "jump tables alias s_P / s_R");
    constexpr uint32_t kJU = kChunk / kSegThreads;
    {
        uint32_t jn[kJU];
        uint64_t jb[kJU];
#pragma unroll
        for (uint32_t u = 0; u < kJU; u++) {  // two blocks
            const uint32_t x = tid + u * nt;
            jn[u] = 0;
            jb[u] = 0;
            if (x < cn) {
                const uint32_t n1 = s_nx[x];
                uint64_t b = s_bb[x];
                uint32_t n = n1, c = 1;
                if (n1 < cn) {
                    b += s_bb[n1];
                    n = s_nx[n1];
                    c = 2;
                }
                jn[u] = n | c << 16;
                jb[u] = b;
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kJU; u++) {
            const uint32_t x = tid + u * nt;
            if (x < cn) {
                j_nx[x] = jn[u];
                j_bb[x] = jb[u];
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < kJU; u++) {  // four blocks
            const uint32_t x = tid + u * nt;
            if (x < cn) {
                const uint32_t n = jn[u] & 0xFFFF;
                if (n < cn) {
                    const uint32_t w = j_nx[n];
                    jb[u] += j_bb[n];
                    jn[u] = (w & 0xFFFF) | ((jn[u] >> 16) + (w >> 16)) << 16;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < kJU; u++) {
            const uint32_t x = tid + u * nt;
            if (x < cn) {
                j_nx[x] = jn[u];
                j_bb[x] = jb[u];
            }
        }
        __syncthreads();
    }
    for (uint32_t c = tid; c < Wc; c += nt) {
        uint32_t e = c, cnt = 0;
        uint64_t by = 0;
        while (e < cn) {
            const uint32_t v = j_nx[e];
            by += j_bb[e];
            cnt += v >> 16;
            e = v & 0xFFFF;
        }
        const uint64_t t = (uint64_t)k * a.seg_look + c;
        // 0xFFFFFFFF: the exit is beyond the u16 range (resolve then walks next[])
        a.tab_exit[t] = c >= cn ? (uint32_t)ce : (e == 0xFFFF ? 0xFFFFFFFFu : (uint32_t)(cs + e));
        a.tab_cnt[t] = cnt;
        a.tab_bytes[t] = by;
    }
    PHASE_MARK(5);
    PHASE_MARK(6);
}

// k_seg: workgroups [0, max_chunks) segment chunk x; with the fused bloom, workgroups past them fill
// bitmap slice x - max_chunks from the slots k_facts binned (independent of the segmentation: both
// only need k_facts, and both are latency-bound, so they share the CUs in one launch).
__global__ __launch_bounds__(kSegThreads, SDB_SEG_WAVES) void k_seg(SstSet P) {
    const EncodeArgs a = make_args(P, blockIdx.y);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (blockIdx.x < P.max_chunks) {
        if (blockIdx.x < a.nchunks) seg_chunk(a, smem, blockIdx.x);
    } else if (a.bloom_fused && blockIdx.x - P.max_chunks < a.bpl.nslices) {
        bloom_fill_slice(blockIdx.x - P.max_chunks, a.key_bytes, a.key_off, a.n, a.bpl, a.bq, a.bloom_out,
                         a.bloom_len, (uint32_t *)smem);
    }
}

// ------------------------------------------------------------------------------------------------
// K2 group: compose the chunk transfer tables of each group of a.group consecutive chunks (one
// workgroup per group): for every candidate entry offset o < W into the group's first chunk, the
// exit offset into the chunk after the group and the blocks / bytes on the way.  k_enum then walks
// the group tables and its own group's chunk tables from entry 0 (<= ~2 sqrt(nchunks) steps).
// Workgroup 0 also reduces the per-chunk SstStats / error partials and initialises the device
// state the later kernels use.  When the tables cannot describe the chain (blocks longer than
// the staged lookahead) or do not fit k_enum's LDS, workgroup 0 walks next() serially instead and
// writes every chunk's anchors (mode 0).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kGroupThreads) void k_group(SstSet P) {
    const EncodeArgs a = make_args(P, blockIdx.y);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t s_W;
    __shared__ unsigned long long s_err;
    __shared__ uint64_t s_stat[5][kGroupThreads / 64];
    const uint32_t K = a.nchunks, g = blockIdx.x, G = a.group, ngroups = (K + G - 1) / G;
    if (g >= ngroups) return;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (blockIdx.y == 0) PHASE_MARK_AT(1023, 5);
    if (tid == 0) {
        s_W = 0;
        s_err = ~0ull;
    }
    __syncthreads();
    {
        uint32_t m = 0;
        unsigned long long em = ~0ull;
        uint64_t st[5] = {0, 0, 0, 0, 0};
        for (uint32_t q = tid; q < K; q += nt) {
            const uint32_t w = a.wmax_part[q];
            m = w > m ? w : m;
        }
        if (g == 0) {
            for (uint32_t q = tid; q < a.nfacts; q += nt) {
                const unsigned long long ep = a.err_part[q];
                em = ep < em ? ep : em;
#pragma unroll
                for (int f = 0; f < 5; f++) st[f] += a.stat_part[5 * (uint64_t)q + f];
            }
        }
        m = wave_max(m);
        if (lane_id() == 0) atomicMax(&s_W, m);
        if (g == 0) {
            if (em != ~0ull) atomicMin(&s_err, em);
#pragma unroll
            for (int f = 0; f < 5; f++) {
                const uint64_t t = wave_sum(st[f]);
                if (lane_id() == 0) s_stat[f][tid >> 6] = t;
            }
        }
    }
    __syncthreads();
    const uint32_t W = s_W;
    // mode 1: the tables describe the chain and k_enum stages its walk in LDS; mode 2: the same walk
    // straight from HBM (tables too large for k_enum's LDS: blocks of 16 KiB and more); mode 0: blocks
    // longer than the staged lookahead, anchors by a serial walk of next()
    const bool fast = W >= 1 && W <= a.seg_look;
    const bool enum_lds = (uint64_t)W * (ngroups + G) * 16 + 64 <= kEnumTabLds;
    if (g == 0 && tid == 0) {
        // device state for k_enum / k_emit (this kernel runs alone on the stream)
        *a.wmax = W;
        *a.err = s_err;
        *a.slow_count = 0;
        *a.big_count = 0;
        a.done[0] = 0;
        a.done[1] = 0;
        *a.mode = fast ? (enum_lds ? 1u : 2u) : 0u;
        sdb_sst_summary *sm = a.summary;
        uint64_t t[5];
        for (int f = 0; f < 5; f++) {
            t[f] = 0;
            for (uint32_t q = 0; q < nt / 64; q++) t[f] += s_stat[f][q];
        }
        sm->raw_key_size = t[0];
        sm->raw_val_size = t[1];
        sm->num_puts = t[2];
        sm->num_deletes = t[3];
        sm->num_merges = t[4];
        sm->num_entries = a.n;
        sm->bloom_len = 0;
        sm->num_probes = 0;
        sm->filter_built = 0;
        sm->status = 0;
        sm->max_block_entries = 0;
        sm->first_error_entry = ~0ull;
        if (!fast) {
            // serial walk of the block chain (one next() step per block), anchors for every chunk
            uint64_t e = 0, blk = 0, by = 0;
            for (uint32_t k = 0; k < K; k++) {
                const uint64_t cs = (uint64_t)k * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
                a.anchor_e[k] = (uint32_t)e;
                a.anchor_blk[k] = (uint32_t)blk;
                a.anchor_byte[k] = by;
                while (e < ce) {
                    by += a.bbytes[e];
                    blk++;
                    e = a.next[e];
                }
            }
            a.anchor_e[K] = (uint32_t)a.n;
            a.anchor_blk[K] = (uint32_t)blk;
            a.anchor_byte[K] = by;
            sm->num_blocks = blk;
            sm->data_len = by;
            if (blk > a.block_cap || by > a.data_cap) report_error(a.err, 0, SDB_INVALID_ARGUMENT);
        }
    }
    if (!fast) return;
    // this group's chunk tables -> LDS (exit offsets clamped into [0, W): candidates past a chunk's
    // own bound are never entry points, their stale slots only need to stay in range)
    const uint32_t k0 = g * G, k1 = k0 + G < K ? k0 + G : K, nk = k1 - k0;
    if ((uint64_t)nk * W * 14 + 64 > kGroupLds) {
        // too large for LDS: each candidate walks the chunk tables in HBM (the same clamping)
        for (uint32_t o = tid; o < W; o += nt) {
            uint32_t e = o, c = 0;
            uint64_t b = 0;
            for (uint32_t j = 0; j < nk; j++) {
                const uint32_t k = k0 + j;
                const uint64_t cs = (uint64_t)k * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
                uint32_t x = 0;
                if (cs + e < ce) {
                    const uint64_t t = (uint64_t)k * a.seg_look + e;
                    const uint32_t te = a.tab_exit[t];
                    x = te >= ce && te - ce < W ? (uint32_t)(te - ce) : W - 1;
                    c += a.tab_cnt[t];
                    b += a.tab_bytes[t];
                }
                e = x;
            }
            const uint64_t t = (uint64_t)g * a.seg_look + o;
            a.gtab_exit[t] = e;
            a.gtab_cnt[t] = c;
            a.gtab_bytes[t] = b;
        }
        return;
    }
    uint16_t *ex = (uint16_t *)smem;                                 // nk x W
    uint32_t *cn_ = (uint32_t *)(smem + ((2 * nk * W + 15) & ~15u)); // nk x W
    uint64_t *by_ = (uint64_t *)((uint8_t *)cn_ + ((4 * nk * W + 15) & ~15u));
    for (uint32_t idx = tid; idx < nk * W; idx += nt) {
        const uint32_t j = idx / W, o = idx - j * W, k = k0 + j;
        const uint64_t cs = (uint64_t)k * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
        uint32_t x = 0, c = 0;
        uint64_t b = 0;
        if (cs + o < ce) {
            const uint64_t t = (uint64_t)k * a.seg_look + o;
            const uint32_t te = a.tab_exit[t];
            x = te >= ce && te - ce < W ? (uint32_t)(te - ce) : W - 1;
            c = a.tab_cnt[t];
            b = a.tab_bytes[t];
        }
        ex[idx] = (uint16_t)x;
        cn_[idx] = c;
        by_[idx] = b;
    }
    __syncthreads();
    for (uint32_t o = tid; o < W; o += nt) {
        uint32_t e = o, c = 0;
        uint64_t b = 0;
        for (uint32_t j = 0; j < nk; j++) {
            c += cn_[j * W + e];
            b += by_[j * W + e];
            e = ex[j * W + e];
        }
        const uint64_t t = (uint64_t)g * a.seg_look + o;
        a.gtab_exit[t] = e;
        a.gtab_cnt[t] = c;
        a.gtab_bytes[t] = b;
    }
}

// ------------------------------------------------------------------------------------------------
// K5: emit
// ------------------------------------------------------------------------------------------------
struct RowInfo {
    uint64_t key_src;   // global byte offset (into key_bytes) of the key suffix
    uint64_t val_src;   // global byte offset (into val_bytes) of the value
    uint32_t suf, vlen; // suffix / value length
    uint32_t shared;
    uint32_t row_off;   // offset of the row in the block
    uint32_t size;
    uint8_t flags;
};

// Encode the row described by (r, seq, ts) into `dst` (LDS or global) byte by byte for the small
// fields; values and key suffixes come from `ksrc`/`vsrc` (LDS staging or global).
template <int V>
SDB_DEV void write_row_small(uint8_t *dst, const RowInfo &r, uint64_t seq, int64_t ets, int64_t cts,
                             uint32_t *hdr_len_out) {
    uint32_t p = 0;
    if (V == 2) {  // SstRowCodecV2::encode (row_codec_v2.rs:127-169)
        uint32_t vals[3] = {r.shared, r.suf, r.vlen};
#pragma unroll
        for (int f = 0; f < 3; f++) {
            uint32_t x = vals[f];
            while (x >= 0x80) {
                dst[p++] = (uint8_t)(x | 0x80);
                x >>= 7;
            }
            dst[p++] = (uint8_t)x;
        }
    } else {  // SstRowCodecV0::encode (row.rs:159-198)
        dst[p++] = (uint8_t)(r.shared >> 8);
        dst[p++] = (uint8_t)r.shared;
        dst[p++] = (uint8_t)(r.suf >> 8);
        dst[p++] = (uint8_t)r.suf;
    }
    *hdr_len_out = p;
    // trailer after key suffix (+ value for V2)
    uint32_t t = p + r.suf + (V == 2 ? r.vlen : 0);
#pragma unroll
    for (int q = 0; q < 8; q++) dst[t++] = (uint8_t)(seq >> (56 - 8 * q));
    dst[t++] = r.flags;
    if (r.flags & SDB_FLAG_HAS_EXPIRE_TS)
#pragma unroll
        for (int q = 0; q < 8; q++) dst[t++] = (uint8_t)((uint64_t)ets >> (56 - 8 * q));
    if (r.flags & SDB_FLAG_HAS_CREATE_TS)
#pragma unroll
        for (int q = 0; q < 8; q++) dst[t++] = (uint8_t)((uint64_t)cts >> (56 - 8 * q));
    if (V == 1 && !(r.flags & SDB_FLAG_TOMBSTONE)) {
        dst[t++] = (uint8_t)(r.vlen >> 24);
        dst[t++] = (uint8_t)(r.vlen >> 16);
        dst[t++] = (uint8_t)(r.vlen >> 8);
        dst[t++] = (uint8_t)r.vlen;
    }
}

// Byte-granular copy between LDS regions with dword realignment (dst, src arbitrary alignment).
SDB_DEV void lds_copy(uint8_t *dst, const uint8_t *src, uint32_t n) {
    uint32_t i = 0;
    while (i < n && (((uintptr_t)(dst + i)) & 3)) {
        dst[i] = src[i];
        i++;
    }
    if (i + 4 <= n) {
        uintptr_t sa = (uintptr_t)(src + i);
        uint32_t sh = (uint32_t)(sa & 3);
        const uint32_t *sw = (const uint32_t *)(sa - sh);
        uint32_t *dw = (uint32_t *)(dst + i);
        uint32_t nw = (n - i) >> 2;
        if (sh == 0) {
            for (uint32_t w = 0; w < nw; w++) dw[w] = sw[w];
        } else {
            uint32_t lo = sw[0];
            for (uint32_t w = 0; w < nw; w++) {
                uint32_t hi = sw[w + 1];
                dw[w] = __builtin_amdgcn_alignbyte(hi, lo, sh);
                lo = hi;
            }
        }
        i += nw * 4;
    }
    while (i < n) {
        dst[i] = src[i];
        i++;
    }
}

SDB_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stage global bytes [g0, g1) into LDS so that stage[x - (g0 & ~15)] = g[x].  One wave, 16-byte
// loads (every loaded 16-byte granule holds at least one requested byte).
SDB_DEV void wave_stage(uint8_t *stage, const uint8_t *g, uint64_t g0, uint64_t g1) {
    if (g1 <= g0) return;
    uint64_t a0 = g0 & ~15ull, a1 = (g1 + 15) & ~15ull;
    uint32_t nchunk = (uint32_t)((a1 - a0) >> 4);
    const uint4 *src = (const uint4 *)(g + a0);
    uint4 *dst = (uint4 *)stage;
    for (uint32_t c = lane_id(); c < nchunk; c += 64) dst[c] = src[c];
}

// Store LDS image bytes [0, len) to global [dst, dst+len); image byte 0 sits at img + (dst & 15).
SDB_DEV void wave_store(uint8_t *gdst, const uint8_t *img, uint64_t len) {
    uintptr_t d0 = (uintptr_t)gdst, d1 = d0 + len;
    uintptr_t a0 = d0 & ~(uintptr_t)15, a1 = (d1 + 15) & ~(uintptr_t)15;
    uint32_t nchunk = (uint32_t)((a1 - a0) >> 4);
    for (uint32_t c = lane_id(); c < nchunk; c += 64) {
        uintptr_t ga = a0 + 16 * (uintptr_t)c;
        const uint8_t *li = img + 16 * c;
        if (ga >= d0 && ga + 16 <= d1) {
            *(uint4 *)ga = *(const uint4 *)li;
        } else {
            for (int q = 0; q < 16; q++)
                if (ga + q >= d0 && ga + q < d1) ((uint8_t *)ga)[q] = li[q];
        }
    }
}

// Blocks k_emit assembles in its per-wave LDS image; the rest take the workgroup slow path.
SDB_DEV bool emit_fast(const BlockDesc &d) {
    const uint32_t ne = d.e - d.s;
    const uint64_t va = d.vs & ~15ull, ka = d.ks & ~15ull;
    const uint32_t nv16 = d.ve > d.vs ? (uint32_t)((d.ve - va + 15) >> 4) : 0;
    const uint32_t nk16 = (uint32_t)((d.ke - ka + 15) >> 4);
    return ne <= 64 && d.bb + 64 <= kImgCap && nv16 <= kStageCap / 16 && nk16 <= kKeyStageCap / 16;
}

// ------------------------------------------------------------------------------------------------
// K5a: enumerate the blocks of each chunk (binary lifting over next()) -> BlockMeta offsets and the
//      per-block descriptors the emitter streams.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kEnumThreads) void k_enum(SstSet P) {
    const EncodeArgs a = make_args(P, blockIdx.y);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t s_anc[4];  // entry point, first block, first byte, blocks of this chunk
    const uint32_t k = blockIdx.x, K = a.nchunks;
    if (k >= K) return;
    if (*a.err != ~0ull) return;
    const uint64_t cs = (uint64_t)k * kChunk;
    const uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
    const uint32_t cn = (uint32_t)(ce - cs);
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    PHASE_MARK_E(0);
    uint32_t *bl_s = (uint32_t *)smem;
    uint32_t *bl_b = bl_s + kChunk;
    uint64_t *bl_o = (uint64_t *)(bl_b + kChunk);
    uint16_t *lv = (uint16_t *)(bl_o + kChunk);
    // next() and the block bytes of every chunk entry are independent of the entry point: their loads
    // go out now and land while the tables are walked (bl_b holds the bytes by entry until the scan)
    constexpr uint32_t kU = (kChunk + kEnumThreads - 1) / kEnumThreads;
    uint32_t nx[kU], eb[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
        const uint32_t x = u * nt + tid;
        nx[u] = x < cn ? a.next[cs + x] : 0;
        eb[u] = x < cn ? a.bbytes[cs + x] : 0;
    }
    if (*a.mode == 2) {
        // the same walk as below, one thread straight through the tables in HBM (they do not fit LDS)
        if (tid == 0) {
            const uint32_t W = *a.wmax, G = a.group, g = k / G, k0 = g * G;
            uint32_t e = 0;
            uint64_t blk = 0, by = 0;
            for (uint32_t q = 0; q < g; q++) {
                const uint64_t t = (uint64_t)q * a.seg_look + e;
                blk += a.gtab_cnt[t];
                by += a.gtab_bytes[t];
                const uint32_t x = a.gtab_exit[t];
                e = x < W ? x : W - 1;
            }
            for (uint32_t kk = k0; kk < k; kk++) {
                const uint64_t ccs = (uint64_t)kk * kChunk, cce = ccs + kChunk < a.n ? ccs + kChunk : a.n;
                uint32_t x = 0;
                if (ccs + e < cce) {
                    const uint64_t t = (uint64_t)kk * a.seg_look + e;
                    const uint32_t te = a.tab_exit[t];
                    x = te >= cce ? te - (uint32_t)cce : 0;
                    blk += a.tab_cnt[t];
                    by += a.tab_bytes[t];
                }
                e = x < W ? x : W - 1;
            }
            uint32_t cn = 0;
            uint64_t cb = 0;
            if (cs + e < ce) {
                const uint64_t t = (uint64_t)k * a.seg_look + e;
                cn = a.tab_cnt[t];
                cb = a.tab_bytes[t];
            }
            s_anc[0] = cs + e;
            s_anc[1] = blk;
            s_anc[2] = by;
            s_anc[3] = cn;
            if (k + 1 == K) {
                const uint64_t tb = blk + cn, ty = by + cb;
                a.anchor_blk[K] = (uint32_t)tb;
                a.anchor_byte[K] = ty;
                a.anchor_e[K] = (uint32_t)a.n;
                a.summary->num_blocks = tb;
                a.summary->data_len = ty;
                if (tb > a.block_cap || ty > a.data_cap) report_error(a.err, 0, SDB_INVALID_ARGUMENT);
            }
        }
        __syncthreads();
    } else if (*a.mode) {
        // walk the group tables of the groups before this chunk's, then this group's chunk tables
        // (k's own last: its block count), from entry 0.  Tables -> LDS first (one batch of loads).
        const uint32_t W = *a.wmax, G = a.group, g = k / G, k0 = g * G, nc = k - k0 + 1;
        const uint32_t ntab = g + nc;
        const uint32_t tb4 = (4 * ntab * W + 15) & ~15u;
        uint32_t *t_ex = (uint32_t *)lv;                 // ntab x W each
        uint32_t *t_cn = (uint32_t *)((uint8_t *)lv + tb4);
        uint64_t *t_by = (uint64_t *)((uint8_t *)lv + 2 * tb4);
        constexpr uint32_t kU = 8;  // table entries per thread per batch: all loads issued first
        for (uint32_t base = 0; base < ntab * W; base += kU * nt) {
            uint32_t x[kU], c[kU];
            uint64_t b[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t idx = base + u * nt + tid;
                x[u] = c[u] = 0;
                b[u] = 0;
                if (idx >= ntab * W) continue;
                const uint32_t q = idx / W, o = idx - q * W;
                if (q < g) {
                    const uint64_t t = (uint64_t)q * a.seg_look + o;
                    x[u] = a.gtab_exit[t];
                    c[u] = a.gtab_cnt[t];
                    b[u] = a.gtab_bytes[t];
                } else {
                    const uint32_t kk = k0 + (q - g);
                    const uint64_t ccs = (uint64_t)kk * kChunk, cce = ccs + kChunk < a.n ? ccs + kChunk : a.n;
                    if (ccs + o < cce) {
                        const uint64_t t = (uint64_t)kk * a.seg_look + o;
                        const uint32_t te = a.tab_exit[t];
                        x[u] = te >= cce ? te - (uint32_t)cce : 0;
                        c[u] = a.tab_cnt[t];
                        b[u] = a.tab_bytes[t];
                    }
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t idx = base + u * nt + tid;
                if (idx >= ntab * W) continue;
                t_ex[idx] = x[u] < W ? x[u] : W - 1;
                t_cn[idx] = c[u];
                t_by[idx] = b[u];
            }
        }
        __syncthreads();
        PHASE_MARK_E(1);
        if (tid == 0) {
            uint32_t e = 0;
            uint64_t blk = 0, by = 0;
            for (uint32_t q = 0; q + 1 < ntab; q++) {
                blk += t_cn[q * W + e];
                by += t_by[q * W + e];
                e = t_ex[q * W + e];
            }
            const uint32_t q = ntab - 1;  // chunk k itself
            s_anc[0] = cs + e;
            s_anc[1] = blk;
            s_anc[2] = by;
            s_anc[3] = cs + e < ce ? t_cn[q * W + e] : 0;
            if (k + 1 == K) {  // totals (the chain's last blocks are this chunk's)
                const uint64_t tb = blk + s_anc[3], ty = by + (cs + e < ce ? t_by[q * W + e] : 0);
                a.anchor_blk[K] = (uint32_t)tb;
                a.anchor_byte[K] = ty;
                a.anchor_e[K] = (uint32_t)a.n;
                a.summary->num_blocks = tb;
                a.summary->data_len = ty;
                if (tb > a.block_cap || ty > a.data_cap) report_error(a.err, 0, SDB_INVALID_ARGUMENT);
            }
        }
        __syncthreads();
    } else if (tid == 0) {
        s_anc[0] = a.anchor_e[k];
        s_anc[1] = a.anchor_blk[k];
        s_anc[2] = a.anchor_byte[k];
        s_anc[3] = a.anchor_blk[k + 1] - a.anchor_blk[k];
    }
    __syncthreads();
    PHASE_MARK_E(2);
    const uint64_t e0 = s_anc[0];
    const uint32_t blk0 = (uint32_t)s_anc[1];
    const uint32_t nb = (uint32_t)s_anc[3];
    const uint64_t byte0 = s_anc[2];
    if (blk0 + (uint64_t)nb > a.block_cap) {  // capacity: the last chunk reports it
        if (tid == 0) report_error(a.err, 0, SDB_INVALID_ARGUMENT);
        return;
    }
    if (k + 1 == K && tid == 0) {
        a.out_block_off[blk0 + nb] = a.anchor_byte[K];
        a.out_block_first[blk0 + nb] = (uint32_t)a.n;
    }
    if (!nb) return;
    uint32_t levels = 1;
    while ((1u << levels) < nb) levels++;
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
        const uint32_t x = u * nt + tid;
        if (x < cn) {
            lv[x] = (uint16_t)(nx[u] >= ce ? cn : (uint32_t)(nx[u] - cs));
            bl_b[x] = eb[u];  // by entry for now
        }
    }
    __syncthreads();
    PHASE_MARK_E(3);
    for (uint32_t j = 1; j < levels; j++) {
        uint16_t *src = lv + (uint64_t)(j - 1) * kChunk, *dst = lv + (uint64_t)j * kChunk;
        for (uint32_t x = tid; x < cn; x += nt) {
            uint16_t y = src[x];
            dst[x] = (y >= cn) ? (uint16_t)cn : src[y];
        }
        __syncthreads();
    }
    uint32_t bx[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
        const uint32_t t = u * nt + tid;
        bx[u] = 0;
        if (t < nb) {
            uint32_t x = (uint32_t)(e0 - cs);
            for (uint32_t j = 0; j < levels; j++)
                if ((t >> j) & 1) x = lv[(uint64_t)j * kChunk + x];
            bl_s[t] = (uint32_t)cs + x;
            bx[u] = bl_b[x];
        }
    }
    __syncthreads();  // every by-entry read of bl_b is done: it becomes by block
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
        const uint32_t t = u * nt + tid;
        if (t < nb) bl_b[t] = bx[u];
    }
    __syncthreads();
    PHASE_MARK_E(4);
    if (tid < 64) {
        uint64_t carry = byte0;
        for (uint32_t g = 0; g < nb; g += 64) {
            uint32_t t = g + tid;
            uint64_t v = t < nb ? bl_b[t] : 0;
            uint64_t inc = wave_incl_scan(v);
            if (t < nb) bl_o[t] = carry + inc - v;
            carry += wave_readlane(inc, 63);
        }
    }
    __shared__ uint32_t s_nbig, s_bigbase;
    uint32_t *big_local = (uint32_t *)lv;  // the lifting levels are done: this chunk's piece-path blocks
    if (tid == 0) s_nbig = 0;
    __syncthreads();
    for (uint32_t t = tid; t < nb; t += nt) {
        const uint64_t s = bl_s[t], e = t + 1 < nb ? bl_s[t + 1] : a.next[s];
        uint32_t blk = blk0 + t;
        a.out_block_off[blk] = bl_o[t];
        a.out_block_first[blk] = (uint32_t)s;
        BlockDesc d;
        d.s = (uint32_t)s;
        d.e = (uint32_t)e;
        d.off = bl_o[t];
        d.vs = a.val_off[s];
        d.ve = a.val_off[e];
        d.ks = a.key_off[s];
        d.ke = a.key_off[e];
        d.bb = bl_b[t];
        d.pad = 0;
        if (!emit_fast(d)) {
            // too big for one wave image: k_emit's piece path, unless a row is too large for a piece
            // (then the workgroup path, marked pad = 1)
            uint32_t h = 0;
            for (uint64_t q = s / kChunk; q <= (e - 1) / kChunk; q++) h |= a.huge_part[q];
            if (h) {
                d.pad = 1;
                a.slow_list[atomicAdd(a.slow_count, 1u)] = blk;
            } else {
                big_local[atomicAdd(&s_nbig, 1u)] = blk;  // LDS: one global reservation per chunk below
            }
        }
        a.desc[blk] = d;
    }
    __syncthreads();
    const uint32_t nbig = s_nbig;
    if (nbig) {  // (a global atomic per big block serialised on the counter: 65 us per SST at 8 KiB blocks)
        if (tid == 0) s_bigbase = atomicAdd(a.big_count, nbig);
        __syncthreads();
        for (uint32_t i = tid; i < nbig; i += nt) a.big_list[s_bigbase + i] = big_local[i];
    }
    PHASE_MARK_E(5);
}

// ------------------------------------------------------------------------------------------------
// K2' anchor (the encode's k_group + the table walks k_enum did per chunk): one workgroup per SST.
//   1. workgroup 0's part of k_group: the SstStats / error partials, the longest candidate block (W)
//      and the device state of the later kernels;
//   2. every chunk's anchor (entry point, first block, first byte) from k_seg's chunk transfer tables,
//      staged in LDS (u16 exit, u16 blocks, u64 bytes): composed per group of a.group chunks (a lane per
//      (group, candidate)), the groups walked from entry 0 (one lane), then each group's chunks from its
//      entry (a lane per group) — about 3 sqrt(nchunks) dependent LDS steps for the SST, where every
//      k_enum workgroup used to stage its own group tables and walk them.  Tables over the LDS are
//      walked the same way straight from HBM.
//   Mode 0 (blocks longer than the lookahead): the serial walk of next(), as k_group.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kAnchorThreads = 1024;
constexpr uint32_t kAnchorLds = 148 * 1024;

__global__ __launch_bounds__(kAnchorThreads) void k_anchor(SstSet P) {
    const EncodeArgs a = make_args(P, blockIdx.y);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t s_W;
    __shared__ unsigned long long s_err;
    __shared__ uint64_t s_stat[5][kAnchorThreads / 64];
    const uint32_t K = a.nchunks, G = a.group, ngroups = (K + G - 1) / G;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (blockIdx.y == 0) PHASE_MARK_AT(1023, 5);
    if (tid == 0) {
        s_W = 0;
        s_err = ~0ull;
    }
    __syncthreads();
    {
        uint32_t m = 0;
        unsigned long long em = ~0ull;
        uint64_t st[5] = {0, 0, 0, 0, 0};
        for (uint32_t q = tid; q < K; q += nt) {
            const uint32_t w = a.wmax_part[q];
            m = w > m ? w : m;
        }
        for (uint32_t q = tid; q < a.nfacts; q += nt) {
            const unsigned long long ep = a.err_part[q];
            em = ep < em ? ep : em;
#pragma unroll
            for (int f = 0; f < 5; f++) st[f] += a.stat_part[5 * (uint64_t)q + f];
        }
        m = wave_max(m);
        if (lane_id() == 0) atomicMax(&s_W, m);
        if (em != ~0ull) atomicMin(&s_err, em);
#pragma unroll
        for (int f = 0; f < 5; f++) {
            const uint64_t t = wave_sum(st[f]);
            if (lane_id() == 0) s_stat[f][tid >> 6] = t;
        }
    }
    __syncthreads();
    if (blockIdx.y == 0) PHASE_MARK_AT(1023, 0);
    const uint32_t W = s_W;
    const bool fast = W >= 1 && W <= a.seg_look;
    sdb_sst_summary *sm = a.summary;
    if (tid == 0) {
        *a.wmax = W;
        *a.err = s_err;
        *a.slow_count = 0;
        *a.big_count = 0;
        a.done[0] = 0;
        a.done[1] = 0;
        *a.mode = fast ? 1u : 0u;
        uint64_t t[5];
        for (int f = 0; f < 5; f++) {
            t[f] = 0;
            for (uint32_t q = 0; q < nt / 64; q++) t[f] += s_stat[f][q];
        }
        sm->raw_key_size = t[0];
        sm->raw_val_size = t[1];
        sm->num_puts = t[2];
        sm->num_deletes = t[3];
        sm->num_merges = t[4];
        sm->num_entries = a.n;
        sm->bloom_len = 0;
        sm->num_probes = 0;
        sm->filter_built = 0;
        sm->status = 0;
        sm->max_block_entries = 0;
        sm->first_error_entry = ~0ull;
    }
    uint64_t tb = 0, ty = 0;  // the chain's blocks and bytes (thread 0)
    if (!fast) {
        if (tid == 0) {  // serial walk of the block chain (one next() step per block)
            uint64_t e = 0;
            for (uint32_t k = 0; k < K; k++) {
                const uint64_t cs = (uint64_t)k * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
                a.anchor_e[k] = (uint32_t)e;
                a.anchor_blk[k] = (uint32_t)tb;
                a.anchor_byte[k] = ty;
                while (e < ce) {
                    ty += a.bbytes[e];
                    tb++;
                    e = a.next[e];
                }
            }
        }
    } else {
        const uint64_t ntab = (uint64_t)K * W, ng = (uint64_t)ngroups * W;
        const uint64_t o_cn = (2 * ntab + 15) & ~15ull, o_by = o_cn + ((2 * ntab + 15) & ~15ull);
        const uint64_t o_gex = o_by + 8 * ntab, o_gcn = o_gex + 4 * ng, o_gby = o_gcn + 4 * ng, o_ent = o_gby + 8 * ng;
        const bool in_lds = o_ent + 16ull * ngroups <= kAnchorLds;
        uint16_t *t_ex = (uint16_t *)smem, *t_cn = (uint16_t *)(smem + o_cn);
        uint64_t *t_by = (uint64_t *)(smem + o_by);
        uint32_t *g_ex = (uint32_t *)(smem + o_gex), *g_cn = (uint32_t *)(smem + o_gcn);
        uint64_t *g_by = (uint64_t *)(smem + o_gby);
        uint32_t *g_ent = (uint32_t *)(smem + o_ent);  // per group: entry offset, blocks before (bytes: g_ent64)
        uint64_t *g_b64 = (uint64_t *)(smem + o_ent + 8ull * ngroups);
        // chunk k's table at candidate o (exit clamped into [0, W): candidates past a chunk's own bound are
        // never entry points, their stale slots only need to stay in range)
        auto tab_hbm = [&](uint32_t k, uint32_t o, uint32_t &x, uint32_t &c, uint64_t &b) {
            const uint64_t cs = (uint64_t)k * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
            x = c = 0;
            b = 0;
            if (cs + o < ce) {
                const uint64_t t = (uint64_t)k * a.seg_look + o;
                const uint32_t te = a.tab_exit[t];
                x = te >= ce && te - ce < W ? (uint32_t)(te - ce) : W - 1;
                c = a.tab_cnt[t];
                b = a.tab_bytes[t];
            }
        };
        auto tab = [&](uint32_t k, uint32_t o, uint32_t &x, uint32_t &c, uint64_t &b) {
            if (in_lds) {
                const uint64_t i = (uint64_t)k * W + o;
                x = t_ex[i];
                c = t_cn[i];
                b = t_by[i];
            } else {
                tab_hbm(k, o, x, c, b);
            }
        };
        if (in_lds) {
            // stage the tables: eight entries per thread in flight, every load unconditional (chunk clamped);
            // entry i's (chunk, candidate) advanced by nt incrementally -- a 64-bit i / W and i % W per entry
            // was half of this kernel's time on one SST
            constexpr uint32_t kU = 8;
            const uint32_t ntab32 = (uint32_t)ntab, qn = nt / W, rn = nt % W;
            uint32_t kk = tid / W, oo = tid % W;
            for (uint32_t base = 0; base < ntab32; base += kU * nt) {
                uint32_t te[kU], tc[kU], ku[kU], ou[kU];
                uint64_t tb[kU];
#pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    ku[u] = kk;
                    ou[u] = oo;
                    oo += rn;
                    kk += qn;
                    if (oo >= W) {
                        oo -= W;
                        kk++;
                    }
                    const uint64_t t = (uint64_t)(ku[u] < K ? ku[u] : K - 1) * a.seg_look + ou[u];
                    te[u] = a.tab_exit[t];
                    tc[u] = a.tab_cnt[t];
                    tb[u] = a.tab_bytes[t];
                }
#pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    const uint32_t i = base + u * nt + tid;
                    if (i >= ntab32) continue;
                    const uint64_t cs = (uint64_t)ku[u] * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
                    const bool in = cs + ou[u] < ce;  // as tab_hbm
                    const uint64_t tx = te[u];
                    t_ex[i] = (uint16_t)(in ? (tx >= ce && tx - ce < W ? (uint32_t)(tx - ce) : W - 1) : 0u);
                    t_cn[i] = (uint16_t)(in ? tc[u] : 0u);  // a block count inside one chunk: <= kChunk
                    t_by[i] = in ? tb[u] : 0ull;
                }
            }
            __syncthreads();
            if (blockIdx.y == 0) PHASE_MARK_AT(1023, 1);
        }
        // tables over the LDS (long SSTs: a 256 MiB compaction output has ~565 chunks): the group tables in
        // LDS, and each group's chunk tables staged into one of kSW per-wave buffers when a wave composes
        // that group, then again when it walks the group's anchors -- every chunk table is read twice, in
        // bulk, instead of one dependent HBM load per chunk on a single lane
        // (its own group size Gs <= G, chosen so that the group tables and a buffer per wave fit beside each
        // other: all 16 waves compose / walk groups at once)
        constexpr uint32_t kSW = kAnchorThreads / 64;
        uint32_t Gs = G, ngs = ngroups;
        uint64_t s_gcn = 0, s_gby = 0, s_gent = 0, s_gb64 = 0, s_buf = 0, wcap = 0, wbytes = 0;
        bool streamed = false;
        for (; !in_lds && Gs >= 1; Gs--) {
            ngs = (K + Gs - 1) / Gs;
            const uint64_t ngw = (uint64_t)ngs * W;
            s_gcn = (4 * ngw + 15) & ~15ull;
            s_gby = s_gcn + ((4 * ngw + 15) & ~15ull);
            s_gent = s_gby + 8 * ngw;
            s_gb64 = s_gent + 8ull * ngs;
            s_buf = (s_gb64 + 8ull * ngs + 15) & ~15ull;
            wcap = (uint64_t)Gs * W;
            wbytes = (wcap * 12 + 15) & ~15ull;
            if (s_buf + kSW * wbytes <= kAnchorLds) {
                streamed = true;
                break;
            }
        }
        if (streamed) {
            uint32_t *sg_ex = (uint32_t *)smem, *sg_cn = (uint32_t *)(smem + s_gcn);
            uint64_t *sg_by = (uint64_t *)(smem + s_gby), *sg_b64 = (uint64_t *)(smem + s_gb64);
            uint32_t *sg_ent = (uint32_t *)(smem + s_gent);
            const uint32_t wv = tid >> 6, ln = tid & 63;
            uint8_t *wb = smem + s_buf + wv * wbytes;
            uint64_t *bb = (uint64_t *)wb;
            uint16_t *bx = (uint16_t *)(wb + 8 * wcap), *bc = bx + wcap;
            // group q's chunk tables -> this wave's buffer (entry (k - q Gs) W + o), eight loads per lane in
            // flight, unconditional (clamped to the group's last entry)
            auto stage_group = [&](uint32_t q) {
                const uint32_t k0 = q * Gs, k1 = (q + 1) * Gs < K ? (q + 1) * Gs : K, ne = (k1 - k0) * W;
                constexpr uint32_t kU = 8;
                const uint32_t q64 = 64 / W, r64 = 64 % W;
                uint32_t kq = ln / W, oq = ln % W;  // (chunk, candidate) of entry i, advanced by 64 (no division)
                for (uint32_t i0 = 0; i0 < ne; i0 += 64 * kU) {
                    uint32_t te[kU], tc[kU], ks[kU], os[kU];
                    uint64_t tbv[kU];
#pragma unroll
                    for (uint32_t u = 0; u < kU; u++) {
                        const uint32_t i = i0 + 64 * u + ln;
                        ks[u] = kq;
                        os[u] = oq;
                        const bool v = i < ne;
                        const uint64_t t = (uint64_t)(k0 + (v ? kq : k1 - k0 - 1)) * a.seg_look + (v ? oq : W - 1);
                        te[u] = a.tab_exit[t];
                        tc[u] = a.tab_cnt[t];
                        tbv[u] = a.tab_bytes[t];
                        oq += r64;
                        kq += q64;
                        if (oq >= W) {
                            oq -= W;
                            kq++;
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < kU; u++) {
                        const uint32_t i = i0 + 64 * u + ln;
                        if (i >= ne) continue;
                        const uint64_t cs = (uint64_t)(k0 + ks[u]) * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
                        const bool in = cs + os[u] < ce;  // as tab_hbm
                        bx[i] = (uint16_t)(in ? (te[u] >= ce && te[u] - ce < W ? (uint32_t)(te[u] - ce) : W - 1) : 0u);
                        bc[i] = (uint16_t)(in ? tc[u] : 0u);
                        bb[i] = in ? tbv[u] : 0ull;
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's LDS writes are done
            };
            for (uint32_t q = wv; q < ngs; q += kSW) {  // group tables: lane per candidate
                stage_group(q);
                const uint32_t nk = ((q + 1) * Gs < K ? (q + 1) * Gs : K) - q * Gs;
                for (uint32_t o = ln; o < W; o += 64) {
                    uint32_t e = o, c = 0;
                    uint64_t b = 0;
                    for (uint32_t j = 0; j < nk; j++) {
                        const uint32_t i = j * W + e;
                        c += bc[i];
                        b += bb[i];
                        e = bx[i];
                    }
                    sg_ex[q * W + o] = e;
                    sg_cn[q * W + o] = c;
                    sg_by[q * W + o] = b;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_s_waitcnt(0xC07F);
            }
            __syncthreads();
            if (blockIdx.y == 0) PHASE_MARK_AT(1023, 1);
            if (tid == 0) {  // the groups from entry 0
                uint32_t e = 0;
                for (uint32_t q = 0; q < ngs; q++) {
                    sg_ent[2 * q] = e;
                    sg_ent[2 * q + 1] = (uint32_t)tb;
                    sg_b64[q] = ty;
                    const uint32_t i = q * W + e;
                    tb += sg_cn[i];
                    ty += sg_by[i];
                    e = sg_ex[i];
                }
            }
            __syncthreads();
            if (blockIdx.y == 0) PHASE_MARK_AT(1023, 2);
            for (uint32_t q = wv; q < ngs; q += kSW) {  // each group's chunks from its entry
                stage_group(q);
                if (ln == 0) {
                    uint32_t e = sg_ent[2 * q];
                    uint64_t blk = sg_ent[2 * q + 1], by = sg_b64[q];
                    const uint32_t k0 = q * Gs, k1 = (q + 1) * Gs < K ? (q + 1) * Gs : K;
                    for (uint32_t k = k0; k < k1; k++) {
                        a.anchor_e[k] = (uint32_t)((uint64_t)k * kChunk + e);
                        a.anchor_blk[k] = (uint32_t)blk;
                        a.anchor_byte[k] = by;
                        const uint32_t i = (k - k0) * W + e;
                        blk += bc[i];
                        by += bb[i];
                        e = bx[i];
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        // group tables: lane per (group, candidate)
        for (uint64_t i = tid; i < ng && in_lds; i += nt) {
            const uint32_t q = (uint32_t)i / W, k1 = (q + 1) * G < K ? (q + 1) * G : K;  // (ng < 2^32 in LDS)
            uint32_t e = (uint32_t)i - q * W, c = 0;
            uint64_t b = 0;
            for (uint32_t k = q * G; k < k1; k++) {
                uint32_t x, cc;
                uint64_t bb;
                tab(k, e, x, cc, bb);
                c += cc;
                b += bb;
                e = x;
            }
            g_ex[i] = e;
            g_cn[i] = c;
            g_by[i] = b;
        }
        __syncthreads();
        if (blockIdx.y == 0 && in_lds) PHASE_MARK_AT(1023, 2);
        if (tid == 0 && !streamed) {  // the groups from entry 0
            uint32_t e = 0;
            for (uint32_t q = 0; q < ngroups; q++) {
                if (in_lds) {
                    g_ent[2 * q] = e;
                    g_ent[2 * q + 1] = (uint32_t)tb;
                    g_b64[q] = ty;
                    const uint64_t i = (uint64_t)q * W + e;
                    tb += g_cn[i];
                    ty += g_by[i];
                    e = g_ex[i];
                } else {  // tables in HBM: this lane walks every chunk (anchors written on the way)
                    const uint32_t k1 = (q + 1) * G < K ? (q + 1) * G : K;
                    for (uint32_t k = q * G; k < k1; k++) {
                        a.anchor_e[k] = (uint32_t)((uint64_t)k * kChunk + e);
                        a.anchor_blk[k] = (uint32_t)tb;
                        a.anchor_byte[k] = ty;
                        uint32_t x, c;
                        uint64_t b;
                        tab_hbm(k, e, x, c, b);
                        tb += c;
                        ty += b;
                        e = x;
                    }
                }
            }
        }
        __syncthreads();
        if (blockIdx.y == 0 && in_lds) PHASE_MARK_AT(1023, 4);
        for (uint32_t q = tid; q < ngroups && in_lds; q += nt) {  // each group's chunks from its entry
            uint32_t e = g_ent[2 * q];
            uint64_t blk = g_ent[2 * q + 1], by = g_b64[q];
            const uint32_t k1 = (q + 1) * G < K ? (q + 1) * G : K;
            for (uint32_t k = q * G; k < k1; k++) {
                a.anchor_e[k] = (uint32_t)((uint64_t)k * kChunk + e);
                a.anchor_blk[k] = (uint32_t)blk;
                a.anchor_byte[k] = by;
                uint32_t x, c;
                uint64_t b;
                tab(k, e, x, c, b);
                blk += c;
                by += b;
                e = x;
            }
        }
    }
    if (blockIdx.y == 0) PHASE_MARK_AT(1023, 3);
    if (tid == 0) {
        a.anchor_e[K] = (uint32_t)a.n;
        a.anchor_blk[K] = (uint32_t)tb;
        a.anchor_byte[K] = ty;
        sm->num_blocks = tb;
        sm->data_len = ty;
        if (tb > a.block_cap || ty > a.data_cap) report_error(a.err, 0, SDB_INVALID_ARGUMENT);
    }
}

// ------------------------------------------------------------------------------------------------
// K5a' blocks (the encode's k_enum, from k_anchor's anchors): per chunk a 256-thread workgroup with
// 16 KiB of LDS (eight per CU): next() and the block bytes of the chunk's entries staged in LDS, the
// chunk's block chain walked from its anchor by one lane, then the blocks in batches of 256: offsets by
// a workgroup scan of their bytes, BlockMeta outputs, descriptors and the big / slow block lists.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kBlkThreads = 256;

__global__ __launch_bounds__(kBlkThreads) void k_blocks(SstSet P) {
    const EncodeArgs a = make_args(P, blockIdx.y);
    __shared__ uint16_t s_nx[kChunk];  // next(cs + x) - cs, clamped to cn
    __shared__ uint32_t s_bb[kChunk];  // block bytes of a block starting at cs + x
    __shared__ uint16_t s_bs[kChunk];  // block t of the chunk starts at cs + s_bs[t]
    __shared__ uint64_t s_w[17];
    __shared__ uint32_t s_nbig, s_bigbase;
    __shared__ uint32_t s_big[kBlkThreads];
    const uint32_t k = blockIdx.x, K = a.nchunks;
    if (k >= K) return;
    if (*a.err != ~0ull) return;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t cs = (uint64_t)k * kChunk, ce = cs + kChunk < a.n ? cs + kChunk : a.n;
    const uint32_t cn = (uint32_t)(ce - cs);
    const uint64_t e0 = a.anchor_e[k], byte0 = a.anchor_byte[k];
    const uint32_t blk0 = a.anchor_blk[k], nb = a.anchor_blk[k + 1] - blk0;
    if (blk0 + (uint64_t)nb > a.block_cap) {  // capacity: k_anchor reports it
        return;
    }
    if (k + 1 == K && tid == 0) {
        a.out_block_off[blk0 + nb] = a.anchor_byte[K];
        a.out_block_first[blk0 + nb] = (uint32_t)a.n;
    }
    if (!nb) return;
    {
        constexpr uint32_t kU = kChunk / kBlkThreads;
        uint32_t nx[kU], eb[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t x = u * nt + tid;
            nx[u] = x < cn ? a.next[cs + x] : 0;
            eb[u] = x < cn ? a.bbytes[cs + x] : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t x = u * nt + tid;
            if (x < cn) {
                s_nx[x] = (uint16_t)(nx[u] >= ce ? cn : (uint32_t)(nx[u] - cs));
                s_bb[x] = eb[u];
            }
        }
    }
    if (tid == 0) s_nbig = 0;
    __syncthreads();
    if (tid == 0) {  // the chain from the anchor: one dependent LDS read per block
        uint32_t x = (uint32_t)(e0 - cs);
        for (uint32_t t = 0; t < nb; t++) {
            s_bs[t] = (uint16_t)x;
            x = s_nx[x];
        }
    }
    __syncthreads();
    uint64_t carry = byte0;
    for (uint32_t b0 = 0; b0 < nb; b0 += nt) {
        const uint32_t t = b0 + tid;
        const bool v = t < nb;
        const uint32_t xs = v ? s_bs[t] : 0;
        const uint32_t bb = v ? s_bb[xs] : 0;
        uint64_t tot;
        const uint64_t off = carry + block_excl_scan_u64(bb, s_w, &tot);
        carry += tot;
        if (v) {
            const uint64_t s = cs + xs, e = t + 1 < nb ? cs + s_bs[t + 1] : a.next[s];
            const uint32_t blk = blk0 + t;
            a.out_block_off[blk] = off;
            a.out_block_first[blk] = (uint32_t)s;
            BlockDesc d;
            d.s = (uint32_t)s;
            d.e = (uint32_t)e;
            d.off = off;
            d.vs = a.val_off[s];
            d.ve = a.val_off[e];
            d.ks = a.key_off[s];
            d.ke = a.key_off[e];
            d.bb = bb;
            d.pad = 0;
            if (!emit_fast(d)) {
                // too big for one wave image: k_emit's piece path, unless a row is too large for a piece
                // (then the workgroup path, marked pad = 1)
                uint32_t h = 0;
                for (uint64_t q = s / kChunk; q <= (e - 1) / kChunk; q++) h |= a.huge_part[q];
                if (h) {
                    d.pad = 1;
                    a.slow_list[atomicAdd(a.slow_count, 1u)] = blk;
                } else {
                    s_big[atomicAdd(&s_nbig, 1u)] = blk;  // one global reservation per batch below
                }
            }
            a.desc[blk] = d;
        }
        __syncthreads();
        const uint32_t nbig = s_nbig;
        if (nbig) {  // (a global atomic per big block serialised on the counter: 65 us per SST at 8 KiB blocks)
            if (tid == 0) s_bigbase = atomicAdd(a.big_count, nbig);
            __syncthreads();
            for (uint32_t i = tid; i < nbig; i += nt) a.big_list[s_bigbase + i] = s_big[i];
            __syncthreads();
            if (tid == 0) s_nbig = 0;
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// K5b: emit.  One wave per block; a workgroup shares the CRC tables (LDS).
//   1. lane = row: row metadata from HBM (offsets, kind, seq, timestamps, LCP), row sizes, a wave
//      scan for the row offsets;
//   2. the row lane writes its row into the wave's LDS image: header / trailer bytes, key suffix and
//      value as dword-aligned interiors (16-byte unaligned HBM loads -> ds_write2_b32) plus <= 3
//      edge bytes each; restart table and count by the restart lanes;
//   3. CRC32: lane l reads 64-byte segment l of the image (image byte 0 = block byte 0, 16-byte
//      aligned), slicing-by-8 per lane, segment l weighted by x^(512 (nseg-1-l)) (4 byte-table
//      lookups), wave XOR, the zero padding of the last segment removed by x^(-8 t);
//   4. 16-byte stores at the block's (unaligned) HBM offset; the < 16-byte tail by one lane.
// ------------------------------------------------------------------------------------------------
SDB_DEV void lds_put_bytes(lu8 *p, uint64_t w, uint32_t n) {  // w little-endian, n <= 8
    for (uint32_t i = 0; i < n; i++) p[i] = (uint8_t)(w >> (8 * i));
}

// lane: image bytes [fa, fa + L) <- global src
SDB_DEV void copy_field(lu8 *img, uint32_t fa, uint32_t L, const uint8_t *src) {
    if (!L) return;
    const uint32_t A0 = (fa + 3) & ~3u, A1 = (fa + L) & ~3u;
    if (A1 <= A0) {  // no whole dword inside: <= 6 bytes
        lds_put_bytes(img + fa, load8(src, L), L);
        return;
    }
    const uint32_t hb = A0 - fa;
    if (hb) lds_put_bytes(img + fa, load8(src, hb), hb);
    const uint8_t *s = src + hb;
    lu32 *d = (lu32 *)(img + A0);
    const uint32_t nd = (A1 - A0) >> 2;
    uint32_t k = 0;
    for (; k + 4 <= nd; k += 4) {
        uint4 v;
        __builtin_memcpy(&v, s + 4 * k, 16);
        d[k] = v.x;
        d[k + 1] = v.y;
        d[k + 2] = v.z;
        d[k + 3] = v.w;
    }
    for (; k < nd; k++) {
        uint32_t v;
        __builtin_memcpy(&v, s + 4 * k, 4);
        d[k] = v;
    }
    const uint32_t tb = fa + L - A1;
    if (tb) lds_put_bytes(img + A1, load8(src + (A1 - fa), tb), tb);
}

// Key-suffix + value copy into the block image.  A row's copy span is [F0, F1): from its key suffix
// (rounded down to a dword) to the end of its value (rounded up).  Each image dword of the span is
// produced by one lane from two aligned LDS dwords + v_alignbyte, reading the key stage for the
// dwords that hold only key bytes and the value stage for all others.  Bytes of those dwords that
// belong to the row's header / trailer, and the <= 3 key bytes that share a dword with value or
// trailer bytes, come out as garbage and are overwritten by the row lane's literal writes, which are
// issued after all copies (DS instructions of one wave execute in order).
//
// The value stage overlaps the image (value byte x of the block is staged at image byte
// x - 64 - (vs & 15) + 64 ... see stage_base): every value is staged at or below its image position
// (a row's header/key/trailer bytes only push it right; the 64-byte guard covers row 0), so copying
// rows in decreasing order never reads a clobbered byte as long as each row is read before it is
// written: a batch of spans of <= 32 dwords reads all of them before writing any; longer spans go
// one row at a time, 64 dwords per pass, passes top-down (a row's image bytes sit >= 52 bytes above
// its staged bytes, so a pass never overwrites the stage of a lower pass).
struct SpanCopy {
    uint32_t a;   // F0 >> 2 | nd << 16: first image dword and dword count of the span
    uint32_t jk;  // leading dwords taken from the key stage
    uint32_t kb;  // LDS byte address (key stage) of image byte F0, as if the key extended left
    uint32_t vb;  // LDS byte address (value stage) of image byte F0, as if the value extended left
};
typedef __attribute__((address_space(3))) SpanCopy lSpanCopy;

SDB_DEV uint32_t span_src(uint32_t j, uint32_t jk, uint32_t kb, uint32_t vb) {
    const uint32_t off = (j < jk ? kb : vb) + 4 * j;
    const lu32 *w = (const lu32 *)(uintptr_t)(off & ~3u);
    return __builtin_amdgcn_alignbyte(w[1], w[0], off & 3);
}

SDB_DEV void copy_spans(lu8 *img, const lSpanCopy *tab, uint32_t ne) {
    const uint32_t l = (uint32_t)lane_id(), half = l >> 5, j0 = l & 31;
    lu32 *dw = (lu32 *)img;
    constexpr uint32_t kB = 4;  // row pairs per batch
    for (uint32_t p0 = 0; p0 < ne; p0 += 2 * kB) {
        uint32_t f0[kB], nd[kB], jk[kB], kb[kB], vb[kB];
        uint32_t mx = 0;
#pragma unroll
        for (uint32_t q = 0; q < kB; q++) {
            const uint32_t i = p0 + 2 * q + half;  // rows in decreasing order
            nd[q] = 0;
            f0[q] = jk[q] = kb[q] = vb[q] = 0;
            if (i < ne) {
                const uint32_t r = ne - 1 - i;
                const u32x4 t = *(const lu128 *)&tab[r];  // one 16-byte broadcast read
                f0[q] = t.x & 0xFFFF;
                nd[q] = t.x >> 16;
                jk[q] = t.y;
                kb[q] = t.z;
                vb[q] = t.w;
            }
            mx = nd[q] > mx ? nd[q] : mx;
        }
        mx = wave_max(mx);
        if (mx <= 32) {
            // every span of the batch fits one pass: all reads, then all writes
            uint32_t v[kB];
#pragma unroll
            for (uint32_t q = 0; q < kB; q++)
                if (j0 < nd[q]) v[q] = span_src(j0, jk[q], kb[q], vb[q]);
#pragma unroll
            for (uint32_t q = 0; q < kB; q++)
                if (j0 < nd[q]) dw[f0[q] + j0] = v[q];
        } else {
            // long spans: one row at a time (decreasing), 64 dwords per pass, passes top-down
            for (uint32_t i = p0; i < p0 + 2 * kB && i < ne; i++) {
                const uint32_t r = ne - 1 - i;
                const uint32_t ta = tab[r].a, rjk = tab[r].jk, rkb = tab[r].kb, rvb = tab[r].vb;
                const uint32_t rf0 = ta & 0xFFFF, rnd = ta >> 16;
                for (uint32_t c = (rnd + 63) >> 6; c-- > 0;) {
                    const uint32_t j = 64 * c + l;
                    uint32_t v = 0;
                    if (j < rnd) v = span_src(j, rjk, rkb, rvb);
                    wave_sync();
                    if (j < rnd) dw[rf0 + j] = v;
                }
            }
        }
    }
}

// Row-lane copy (lane = row) for blocks whose spans fit in registers: every lane first reads the
// aligned source dwords of its span (key run from the key stage, value run from the value stage) into
// registers, and only then does any lane write, so the in-place value stage is never overwritten
// before it is read (rows of one block overlap each other's stage).  One v_alignbyte per image dword
// and about one LDS read + one write per dword, against copy_spans' per-dword table walk and two
// reads.  Returns false (nothing written) when a span is too long; the caller then uses copy_spans.
constexpr uint32_t kRowRegs = 28, kKeyRegs = 6;
SDB_DEV bool copy_rows(lu8 *img, bool row, const SpanCopy &sc) {
    const uint32_t f0 = sc.a & 0xFFFF, nd = row ? sc.a >> 16 : 0;
    const uint32_t jk = row ? (sc.jk < nd ? sc.jk : nd) : 0, nv = nd - jk;
    const uint32_t mk = wave_max(jk), mv = wave_max(nv);
    if (mk + 1 > kKeyRegs || mv + 1 > kRowRegs) return false;
    const uint32_t ks = sc.kb, vs = sc.vb + 4 * jk;  // LDS byte addresses of the two runs' first bytes
    const lu32 *kw = (const lu32 *)(uintptr_t)(ks & ~3u), *vw = (const lu32 *)(uintptr_t)(vs & ~3u);
    uint32_t K[kKeyRegs], W[kRowRegs];
#pragma unroll
    for (uint32_t t = 0; t < kKeyRegs; t++) {
        K[t] = 0;
        if (t <= mk && jk && t <= jk) K[t] = kw[t];
    }
#pragma unroll
    for (uint32_t t = 0; t < kRowRegs; t++) {
        W[t] = 0;
        if (t <= mv && nv && t <= nv) W[t] = vw[t];
    }
    wave_sync();  // every read of the wave is issued (and, in order, done) before the first write
    lu32 *dw = (lu32 *)img + f0;
#pragma unroll
    for (uint32_t t = 0; t + 1 < kKeyRegs; t++)
        if (t < mk && t < jk) dw[t] = __builtin_amdgcn_alignbyte(K[t + 1], K[t], ks & 3);
#pragma unroll
    for (uint32_t t = 0; t + 1 < kRowRegs; t++)
        if (t < mv && t < nv) dw[jk + t] = __builtin_amdgcn_alignbyte(W[t + 1], W[t], vs & 3);
    return true;
}

template <int V>
SDB_DEV uint32_t write_row_hdr_trailer(lu8 *dst, const RowInfo &r, uint64_t seq, int64_t ets, int64_t cts) {
    uint32_t p = 0;
    if (V == 2) {  // SstRowCodecV2::encode (row_codec_v2.rs:127-169)
        if ((r.shared | r.suf | r.vlen) < 0x80) {  // three one-byte varints (the common row)
            dst[0] = (uint8_t)r.shared;
            dst[1] = (uint8_t)r.suf;
            dst[2] = (uint8_t)r.vlen;
            p = 3;
        } else {
            uint32_t vals[3] = {r.shared, r.suf, r.vlen};
#pragma unroll
            for (int f = 0; f < 3; f++) {
                uint32_t x = vals[f];
                while (x >= 0x80) {
                    dst[p++] = (uint8_t)(x | 0x80);
                    x >>= 7;
                }
                dst[p++] = (uint8_t)x;
            }
        }
    } else {  // SstRowCodecV0::encode (row.rs:159-198)
        dst[0] = (uint8_t)(r.shared >> 8);
        dst[1] = (uint8_t)r.shared;
        dst[2] = (uint8_t)(r.suf >> 8);
        dst[3] = (uint8_t)r.suf;
        p = 4;
    }
    const uint32_t h = p;
    uint32_t t = p + r.suf + (V == 2 ? r.vlen : 0);
    lds_put_bytes(dst + t, bswap64(seq), 8);
    t += 8;
    dst[t++] = r.flags;
    if (r.flags & SDB_FLAG_HAS_EXPIRE_TS) {
        lds_put_bytes(dst + t, bswap64((uint64_t)ets), 8);
        t += 8;
    }
    if (r.flags & SDB_FLAG_HAS_CREATE_TS) {
        lds_put_bytes(dst + t, bswap64((uint64_t)cts), 8);
        t += 8;
    }
    if (V == 1 && !(r.flags & SDB_FLAG_TOMBSTONE)) {
        dst[t] = (uint8_t)(r.vlen >> 24);
        dst[t + 1] = (uint8_t)(r.vlen >> 16);
        dst[t + 2] = (uint8_t)(r.vlen >> 8);
        dst[t + 3] = (uint8_t)r.vlen;
    }
    return h;
}

// A block's prefetched data (16-byte granules of its values and keys, lane l holding granules l, l + 64,
// ...) and row metadata (lane = row).
struct EmitData {
    uint4 vg[kStageCap / 1024];
    uint4 kg[kKeyStageCap / 1024];
};
struct EmitMeta {
    uint64_t ko, vo, seq;
    uint64_t pko;  // lane 0: key_off[s - 1] (previous key, index-key rule)
    uint32_t lcp;
    uint32_t kind, mask;
};

SDB_DEV BlockDesc desc_from_lanes(uint32_t dv) {  // lanes 0..13 hold the 14 dwords of a BlockDesc
    uint32_t w[14];
#pragma unroll
    for (int i = 0; i < 14; i++) w[i] = (uint32_t)__builtin_amdgcn_readlane((int)dv, i);
    BlockDesc d;
    d.s = w[0];
    d.e = w[1];
    d.off = w[2] | ((uint64_t)w[3] << 32);
    d.vs = w[4] | ((uint64_t)w[5] << 32);
    d.ve = w[6] | ((uint64_t)w[7] << 32);
    d.ks = w[8] | ((uint64_t)w[9] << 32);
    d.ke = w[10] | ((uint64_t)w[11] << 32);
    d.bb = w[12];
    d.pad = w[13];
    return d;
}
static_assert(sizeof(BlockDesc) == 56, "BlockDesc is 14 dwords");


// A block k_emit skips (not fast, or past the workgroup's share) is emitted as an empty block with its
// stores dropped, so that every iteration issues the same memory instructions (see k_emit).
SDB_DEV BlockDesc desc_or_empty(BlockDesc d, bool live) {
    if (!live) {
        d.e = d.s;
        d.ve = d.vs;
        d.ke = d.ks;
    }
    return d;
}

// Every load is unconditional, from a clamped in-bounds address (lanes past the block re-read its last
// granule; an absent column reads key_off and is masked at use): a load under a branch, even a lane
// predicate, leaves the compiler's vmcnt bookkeeping at the join with the worst case, and k_emit's
// wait for THIS block's data would then also wait for the next block's prefetch.
SDB_DEV void emit_prefetch_data(const EncodeArgs &a, const BlockDesc &d, EmitData &p) {
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t va = d.vs & ~15ull, ka = d.ks & ~15ull;
    const uint32_t nv16 = d.ve > d.vs ? (uint32_t)((d.ve - va + 15) >> 4) : 0;
    const uint32_t nk16 = (uint32_t)((d.ke - ka + 15) >> 4);
    const uint4 *vsrc = nv16 ? (const uint4 *)(a.val_bytes + va) : (const uint4 *)a.key_off;
    const uint4 *ksrc = nk16 ? (const uint4 *)(a.key_bytes + ka) : (const uint4 *)a.key_off;
    const uint32_t vlast = nv16 ? nv16 - 1 : 0, klast = nk16 ? nk16 - 1 : 0;
#pragma unroll
    for (uint32_t q = 0; q < kStageCap / 1024; q++) p.vg[q] = vsrc[64 * q + l < vlast ? 64 * q + l : vlast];
#pragma unroll
    for (uint32_t q = 0; q < kKeyStageCap / 1024; q++) p.kg[q] = ksrc[64 * q + l < klast ? 64 * q + l : klast];
}
SDB_DEV void emit_prefetch_meta(const EncodeArgs &a, const BlockDesc &d, EmitMeta &p) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t ne = d.e - d.s;
    const uint64_t j = d.s + (l < ne ? l : 0);  // rows >= ne read entry s (masked at use)
    p.ko = a.key_off[j];
    p.vo = a.val_off[j];
    p.seq = (a.seq ? a.seq : a.key_off)[j];
    p.lcp = a.lcp[j];
    p.kind = (a.kind ? a.kind : (const uint8_t *)a.key_off)[j];
    p.mask = (a.ts_mask ? a.ts_mask : (const uint8_t *)a.key_off)[j];
    p.pko = a.key_off[d.s > 0 ? d.s - 1 : 0];  // lane 0 uses it when s > 0
}

// 0. the prefetched granules -> the LDS stages: value byte x lands at LDS (img - kStageGuard) + (x - va),
//    i.e. at or below its image position (see copy_spans); keys land in the key stage
SDB_DEV void emit_stage(const BlockDesc &d, const EmitData &p, lu8 *img, lu8 *kst) {
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t va = d.vs & ~15ull, ka = d.ks & ~15ull;
    const uint32_t nv16 = d.ve > d.vs ? (uint32_t)((d.ve - va + 15) >> 4) : 0;
    const uint32_t nk16 = (uint32_t)((d.ke - ka + 15) >> 4);
    const uint32_t vstage = lds_addr((const void *)img) - kStageGuard;
    const uint32_t kstage = lds_addr((const void *)kst);
#ifndef SDB_EXP_EMIT_NOSTAGE  // diagnostic: granules loaded, never staged
#pragma unroll
    for (uint32_t q = 0; q < kStageCap / 1024; q++)
        if (64 * q + l < nv16) *(lu128 *)(uintptr_t)(vstage + 16 * (64 * q + l)) = *(const u32x4 *)&p.vg[q];
#pragma unroll
    for (uint32_t q = 0; q < kKeyStageCap / 1024; q++)
        if (64 * q + l < nk16) *(lu128 *)(uintptr_t)(kstage + 16 * (64 * q + l)) = *(const u32x4 *)&p.kg[q];
#else
    if (l == 0 && p.vg[0].x == 0x12345678u && p.kg[0].y == 0x9abcdefu) img[0] = 1;  // keep the loads
#endif
}

template <int V>
SDB_DEV void emit_block(const EncodeArgs &a, uint32_t blk, const BlockDesc &d, bool live, const EmitMeta &p, lu8 *img,
                        lu8 *kst, lSpanCopy *rtab, const lu32 *crc, uint64_t *ph) {
    WAVE_T(t0);
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t ne = d.e - d.s;
    const uint64_t va = d.vs & ~15ull, ka = d.ks & ~15ull;
    const uint32_t vstage = lds_addr((const void *)img) - kStageGuard;
    const uint32_t kstage = lds_addr((const void *)kst);
    // (0. the stages are written by the caller: emit_stage)
    // 1. row metadata (lane = row)
    const bool row = l < ne;
    const uint64_t ko = p.ko, vo = p.vo, seq = a.seq ? p.seq : 0;
    const uint32_t lcp = p.lcp;
    const uint8_t kind = row && a.kind ? (uint8_t)p.kind : 0, mask = row && a.ts_mask ? (uint8_t)p.mask : 0;
    // timestamps: loaded here, only by a block that carries any (rare; the prefetch keeps its registers)
    int64_t cts = 0, ets = 0;
    if (__ballot(mask & (SDB_TS_CREATE | SDB_TS_EXPIRE))) {
        const uint64_t j = d.s + (row ? l : 0);
        if ((mask & SDB_TS_CREATE) && a.create_ts) cts = a.create_ts[j];
        if ((mask & SDB_TS_EXPIRE) && a.expire_ts) ets = a.expire_ts[j];
        // land them here: a load still pending at the join would make every later write of its
        // registers (reused by the common path) wait for all memory traffic
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    uint32_t prev_klen = 0;
    if (l == 0 && d.s > 0) prev_klen = (uint32_t)(d.ks - p.pko);
    uint64_t ko1 = wave_next_lane(ko), vo1 = wave_next_lane(vo);
    if (l + 1 == ne) {
        ko1 = d.ke;
        vo1 = d.ve;
    }
    const uint32_t klen = row ? (uint32_t)(ko1 - ko) : 0;
    const uint32_t vlen = (row && kind != SDB_KIND_TOMBSTONE) ? (uint32_t)(vo1 - vo) : 0;
    const uint32_t ri = a.restart_interval;
    uint32_t shared = 0;
    if (V == 2 && row) shared = (l % ri == 0) ? 0 : lcp;
    if (V == 1) {  // prefix vs the block's first key (block.rs:117-123), from the key stage
        wave_sync();
        const uint32_t fkl = wave_readlane(klen, 0);
        if (row && l > 0) {
            const lu8 *f = kst + (uint32_t)(d.ks - ka), *c = kst + (uint32_t)(ko - ka);
            const uint32_t mn = fkl < klen ? fkl : klen;
            while (shared < mn && f[shared] == c[shared]) shared++;
        }
    }
    RowInfo r;
    r.shared = shared;
    r.suf = klen - shared;
    r.vlen = vlen;
    r.flags = (uint8_t)((kind == SDB_KIND_MERGE ? SDB_FLAG_MERGE_OPERAND : 0) |
                        (kind == SDB_KIND_TOMBSTONE ? SDB_FLAG_TOMBSTONE : 0) |
                        ((mask & SDB_TS_EXPIRE) ? SDB_FLAG_HAS_EXPIRE_TS : 0) |
                        ((mask & SDB_TS_CREATE) ? SDB_FLAG_HAS_CREATE_TS : 0));
    const uint32_t ts8 = 8u * (((mask & SDB_TS_CREATE) != 0) + ((mask & SDB_TS_EXPIRE) != 0));
    uint32_t size = 0, h = 0;
    if (row) {
        if (V == 2) {
            h = varint_len(shared) + varint_len(r.suf) + varint_len(vlen);
            size = h + r.suf + vlen + 9 + ts8;
        } else {
            h = 4;
            size = 4 + r.suf + 9 + ts8 + (kind == SDB_KIND_TOMBSTONE ? 0 : 4 + vlen);
        }
    }
    r.size = size;
    const uint32_t inc = wave_incl_scan(size);
    const uint32_t row_off = inc - size;
    const uint32_t D = wave_readlane(inc, 63);
    const uint32_t noffs = (V == 2) ? (ne + ri - 1) / ri : ne;
    const uint32_t Lc = D + 2 * noffs + 2;  // CRC input length
    // copy span of the row: key suffix .. value end
    const uint32_t kstart = row_off + h, kend = kstart + r.suf;
    const uint32_t vstart = (V == 2) ? kend : row_off + size - vlen;
    const uint32_t vend = vlen ? vstart + vlen : kend;
    SpanCopy sc{0, 0, 0, 0};
    if (row) {
        const uint32_t F0 = kstart & ~3u, F1 = (vend + 3) & ~3u;
        sc.a = (F0 >> 2) | (((F1 - F0) >> 2) << 16);
        sc.jk = (kend - F0) >> 2;
        sc.kb = kstage + (uint32_t)(ko + shared - ka) - (kstart - F0);
        sc.vb = vstage + (uint32_t)(vo - va) - (vstart - F0);
    }
    WAVE_T(t1);
    wave_sync();  // stages written (DS instructions of one wave complete in order)
    WAVE_T(t2);
    // 2. key suffixes + values: lane = row from registers, or cooperative by the span table
#if defined(SDB_EXP_EMIT_NOCOPY)  // diagnostic: image without key / value bytes
    if (false) {
#elif defined(SDB_EMIT_SPANS)  // the cooperative span copy for every block
    if (true) {
#else
    if (!copy_rows(img, row, sc)) {
#endif
        if (row) {
            rtab[l].a = sc.a;
            rtab[l].jk = sc.jk;
            rtab[l].kb = sc.kb;
            rtab[l].vb = sc.vb;
        }
        wave_sync();
        copy_spans(img, rtab, ne);
    }
    WAVE_T(t3);
    // 3. literals: header, the key bytes sharing a dword with non-key bytes, trailer; then the
    //    restart table, count and the zero padding of the last CRC segment
#ifdef SDB_EXP_EMIT_NOLIT  // diagnostic: no header / trailer / key-edge literals
    if (false) {
#else
    if (row) {
#endif
        write_row_hdr_trailer<V>(img + row_off, r, seq, ets, cts);
        // the <= 3 key bytes that share a dword with value / trailer bytes (predicated, no loop)
        const uint32_t kj = (kend & ~3u) > kstart ? (kend & ~3u) : kstart;
        const lu8 *ksrc = kst + (uint32_t)(ko + shared - ka) - kstart;
#pragma unroll
        for (uint32_t q = 0; q < 3; q++)
            if (kj + q < kend) img[kj + q] = ksrc[kj + q];
    }
    if (V == 2) {
        if (row && l % ri == 0) {
            uint32_t q = l / ri;
            if (row_off > 0xFFFF) report_error(a.err, d.s + l, SDB_LIMIT_EXCEEDED);  // block_v2.rs:195
            img[D + 2 * q] = (uint8_t)(row_off >> 8);
            img[D + 2 * q + 1] = (uint8_t)row_off;
        }
    } else if (row) {
        img[D + 2 * l] = (uint8_t)(row_off >> 8);  // `as u16` (block.rs:163)
        img[D + 2 * l + 1] = (uint8_t)row_off;
    }
    if (l == 0) {
        img[D + 2 * noffs] = (uint8_t)(noffs >> 8);
        img[D + 2 * noffs + 1] = (uint8_t)noffs;
    }
    wave_sync();
    // the value stage below the image is consumed: its 64 bytes become the zero lead-in of the
    // right-aligned CRC segments; crc32fast's init is folded in by inverting image bytes [0, 4)
    // (undone by the store)
    if (l < 16) ((lu32 *)(img - kStageGuard))[l] = 0;
    if (l == 0) ((lu32 *)img)[0] = ~((const lu32 *)img)[0];
    wave_sync();
    WAVE_T(t4);
    // 4. CRC32 (format/sst.rs:541-552) of the image [0, Lc)
#if defined(SDB_EXP_EMIT_NOCRC)  // diagnostic: wrong CRC by design
    const uint32_t crc32 = 0;
#elif defined(SDB_EMIT_CRC_SLICE)
    const uint32_t crc32 = wave_crc_image_ra(img, Lc);
#else
    const uint32_t crc32 = wave_crc_image_mfma<0, kCrcMfmaTreeKiB>(img, Lc);
#endif
    if (l == 0) {
        img[Lc] = (uint8_t)(crc32 >> 24);
        img[Lc + 1] = (uint8_t)(crc32 >> 16);
        img[Lc + 2] = (uint8_t)(crc32 >> 8);
        img[Lc + 3] = (uint8_t)crc32;
        if (live && Lc + 4 != d.bb) report_error(a.err, d.s, SDB_DEVICE_ERROR);  // internal consistency
    }
    wave_sync();
    WAVE_T(t5);
    // 5. store [0, Lc + 4) -> out_data + off: a fixed set of buffer stores (L <= 4096: four 16-byte granule
    //    stores and one tail-byte store per lane), the range check of the buffer descriptor dropping what
    //    lies past the block (or everything: !live) -- no branch, so the count of memory instructions is
    //    the same on every path (see k_emit)
    const uint32_t L = Lc + 4, nfull = L >> 4;
#ifndef SDB_EXP_EMIT_NOSTORE  // diagnostic: the image is never stored
    {
        uint8_t *gdst = a.out_data + d.off;
        const __amdgpu_buffer_rsrc_t rg = wave_rsrc(gdst, live ? nfull << 4 : 0);
        const __amdgpu_buffer_rsrc_t rt = wave_rsrc(gdst, live ? L : 0);
#pragma unroll
        for (uint32_t q = 0; q < kStageCap / 1024; q++) {
            const uint32_t cc = 64 * q + l;
            u32x4 v = ((const lu128 *)img)[cc];
            if (cc == 0) v.x = ~v.x;  // the CRC's init fold
            __builtin_amdgcn_raw_buffer_store_b128(v, rg, (int)(16 * cc), 0, 0);
        }
        const uint32_t tb = (nfull << 4) + l;  // L >= 16: never image bytes [0, 4)
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)img[tb < kImgCap ? tb : 0], rt, (int)(l < (L & 15) ? tb : L), 0, 0);
    }
#else
    if (l == 0 && crc32 == 0x12345678u) a.out_data[d.off] = img[5];
#endif
    WAVE_T(t6);
#ifdef SDB_PHASE_TIMING
    ph[0] += t1 - t0;
    ph[1] += t2 - t1;
    ph[2] += t3 - t2;
    ph[3] += t4 - t3;
    ph[4] += t5 - t4;
    ph[5] += t6 - t5;
    ph[6] += 1;
#endif
    // 6. BlockStats (sst_stats.rs:9-16) and the index key (compute_index_key, utils.rs:198-226): lanes
    //    0..2 store the three counts, lane 0 the index key length, through range-checked buffer stores
    const uint64_t pu = __ballot(row && kind == SDB_KIND_VALUE);
    const uint64_t de = __ballot(row && kind == SDB_KIND_TOMBSTONE);
    const uint64_t me = __ballot(row && kind == SDB_KIND_MERGE);
    {
        const __amdgpu_buffer_rsrc_t rs = wave_rsrc(a.out_block_stats + 3 * (uint64_t)blk, live ? 6 : 0);
        const __amdgpu_buffer_rsrc_t rk = wave_rsrc(a.out_index_key_len + blk, live ? 4 : 0);
        const uint32_t c = (uint32_t)__popcll(l == 0 ? pu : l == 1 ? de : me);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)c, rs, (int)(l < 3 ? 2 * l : 6), 0, 0);
        uint32_t ik = 0;
        if (d.s > 0 && !a.wal) ik = (lcp == prev_klen && prev_klen == klen) ? klen : lcp + 1;
        __builtin_amdgcn_raw_buffer_store_b32(ik, rk, (int)(l == 0 ? 0 : 4), 0, 0);
    }
    wave_sync();
}

// Blocks that do not fit one wave image (over 64 rows or 4 KiB: block sizes of 8-64 KiB) but whose rows
// each fit a piece: the wave assembles the block as consecutive pieces of <= 64 rows and <= 4 KiB, each
// exactly like a small block's rows (metadata lane = row, staged keys / values, row-lane copies, literal
// header / trailer), stores each piece at its offset in the block and chains the CRC32 over the pieces
// (raw(A || B) = raw(A) x^(8 |B|) + raw(B), crc_shift_bytes).  Restart offsets go straight to their
// trailer slots (the trailer's position, D = block bytes - 4 - 2 - 2 noffs, is known from k_seg's block
// size); the trailer is CRC'd last, read back through the image.  No prefetch: the pieces of one block
// keep the wave busy while other waves' loads are in flight.
template <int V>
SDB_DEV void emit_big(const EncodeArgs &a, uint32_t blk, const BlockDesc &d, lu8 *img, lu8 *kst, lSpanCopy *rtab) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t ne = d.e - d.s, ri = a.restart_interval;
    const uint32_t noffs = (V == 2) ? (ne + ri - 1) / ri : ne;
    const uint32_t Lc = d.bb - 4, D = Lc - 2 * noffs - 2;
    uint8_t *gblk = a.out_data + d.off;
    const uint32_t vstage = lds_addr((const void *)img) - kStageGuard, kstage = lds_addr((const void *)kst);
    const uint32_t fkl = (uint32_t)(a.key_off[d.s + 1] - d.ks);  // V1: prefixes against the block's first key
    // a trailer of <= 64 bytes is gathered in the 64 image bytes past 4 KiB that no piece touches, and
    // CRC'd from there; a longer one goes to HBM slot by slot and is read back
    const uint32_t Tl = 2 * noffs + 2;
    const bool tr_lds = Tl <= 64;
    lu8 *tr = img + 4096;
    uint32_t crc = 0, base = 0, pu = 0, de = 0, me = 0, ik = 0;
    for (uint32_t r = 0; r < ne;) {
        const uint32_t nr = ne - r < 64 ? ne - r : 64;
        const bool row = l < nr;
        const uint64_t j = d.s + r + (row ? l : 0);
        const uint64_t ko = a.key_off[j], ko1 = a.key_off[j + 1], vo = a.val_off[j], vo1 = a.val_off[j + 1];
        const uint64_t seq = a.seq ? a.seq[j] : 0;
        const uint32_t lcp = a.lcp[j];
        const uint8_t kind = row && a.kind ? a.kind[j] : 0, mask = row && a.ts_mask ? a.ts_mask[j] : 0;
        const int64_t cts = (mask & SDB_TS_CREATE) ? a.create_ts[j] : 0, ets = (mask & SDB_TS_EXPIRE) ? a.expire_ts[j] : 0;
        const uint32_t klen = row ? (uint32_t)(ko1 - ko) : 0;
        const uint32_t vlen = (row && kind != SDB_KIND_TOMBSTONE) ? (uint32_t)(vo1 - vo) : 0;
        uint32_t shared = 0;
        if (V == 2 && row) shared = ((r + l) % ri == 0) ? 0 : lcp;
        if (V == 1 && row && r + l > 0) {
            const uint32_t mn = fkl < klen ? fkl : klen;
            shared = lcp_bytes(a.key_bytes + d.ks, mn, a.key_bytes + ko, mn);
        }
        if (r == 0 && l == 0 && d.s > 0 && !a.wal) {  // compute_index_key (utils.rs:198-226)
            const uint32_t pkl = (uint32_t)(d.ks - a.key_off[d.s - 1]);
            ik = (lcp == pkl && pkl == klen) ? klen : lcp + 1;
        }
        RowInfo ri_;
        ri_.shared = shared;
        ri_.suf = klen - shared;
        ri_.vlen = vlen;
        ri_.flags = (uint8_t)((kind == SDB_KIND_MERGE ? SDB_FLAG_MERGE_OPERAND : 0) |
                              (kind == SDB_KIND_TOMBSTONE ? SDB_FLAG_TOMBSTONE : 0) |
                              ((mask & SDB_TS_EXPIRE) ? SDB_FLAG_HAS_EXPIRE_TS : 0) |
                              ((mask & SDB_TS_CREATE) ? SDB_FLAG_HAS_CREATE_TS : 0));
        const uint32_t ts8 = 8u * (((mask & SDB_TS_CREATE) != 0) + ((mask & SDB_TS_EXPIRE) != 0));
        uint32_t size = 0, h = 0;
        if (row) {
            if (V == 2) {
                h = varint_len(shared) + varint_len(ri_.suf) + varint_len(vlen);
                size = h + ri_.suf + vlen + 9 + ts8;
            } else {
                h = 4;
                size = 4 + ri_.suf + 9 + ts8 + (kind == SDB_KIND_TOMBSTONE ? 0 : 4 + vlen);
            }
        }
        ri_.size = size;
        const uint32_t inc = wave_incl_scan(size);
        // the piece: the longest prefix of these rows whose bytes, staged values and keys fit
        const uint64_t va = wave_readlane(vo, 0) & ~15ull, ka = wave_readlane(ko, 0) & ~15ull;
        const bool fits = row && inc <= 4096 && (vo1 - va) <= kStageCap && (ko1 - ka) <= kKeyStageCap;
        const uint64_t nofit = __ballot(!fits);
        const uint32_t c = nofit ? (uint32_t)__builtin_ctzll(nofit) : 64u;
        if (c == 0) {  // k_enum routes blocks with rows this large to the workgroup path
            if (l == 0) report_error(a.err, d.s + r, SDB_DEVICE_ERROR);
            return;
        }
        const bool prow = l < c;
        const uint32_t Lp = wave_readlane(inc, c - 1);
        const uint64_t ve = wave_readlane(vo1, c - 1), ke = wave_readlane(ko1, c - 1);
        // stage the piece's values (in place below the image) and keys
        {
            const uint32_t nv16 = ve > va ? (uint32_t)((ve - va + 15) >> 4) : 0, nk16 = (uint32_t)((ke - ka + 15) >> 4);
            const uint4 *vsrc = (const uint4 *)(a.val_bytes + va), *ksrc = (const uint4 *)(a.key_bytes + ka);
            for (uint32_t q = l; q < nv16; q += 64) {
                const uint4 g = vsrc[q];
                u32x4 w;
                w.x = g.x;
                w.y = g.y;
                w.z = g.z;
                w.w = g.w;
                *(lu128 *)(uintptr_t)(vstage + 16 * q) = w;
            }
            for (uint32_t q = l; q < nk16; q += 64) {
                const uint4 g = ksrc[q];
                u32x4 w;
                w.x = g.x;
                w.y = g.y;
                w.z = g.z;
                w.w = g.w;
                *(lu128 *)(uintptr_t)(kstage + 16 * q) = w;
            }
        }
        const uint32_t row_off = inc - size;
        const uint32_t kstart = row_off + h, kend = kstart + ri_.suf;
        const uint32_t vstart = (V == 2) ? kend : row_off + size - vlen;
        const uint32_t vend = vlen ? vstart + vlen : kend;
        SpanCopy sc{0, 0, 0, 0};
        if (prow) {
            const uint32_t F0 = kstart & ~3u, F1 = (vend + 3) & ~3u;
            sc.a = (F0 >> 2) | (((F1 - F0) >> 2) << 16);
            sc.jk = (kend - F0) >> 2;
            sc.kb = kstage + (uint32_t)(ko + shared - ka) - (kstart - F0);
            sc.vb = vstage + (uint32_t)(vo - va) - (vstart - F0);
        }
        wave_sync();
        if (!copy_rows(img, prow, sc)) {
            if (prow) {
                rtab[l].a = sc.a;
                rtab[l].jk = sc.jk;
                rtab[l].kb = sc.kb;
                rtab[l].vb = sc.vb;
            }
            wave_sync();
            copy_spans(img, rtab, c);
        }
        if (prow) {
            write_row_hdr_trailer<V>(img + row_off, ri_, seq, ets, cts);
            const uint32_t kj = (kend & ~3u) > kstart ? (kend & ~3u) : kstart;
            const lu8 *ksrc = kst + (uint32_t)(ko + shared - ka) - kstart;
#pragma unroll
            for (uint32_t q = 0; q < 3; q++)
                if (kj + q < kend) img[kj + q] = ksrc[kj + q];
            // the restart offsets go straight to their trailer slots
            const uint32_t br = base + row_off;
            int q = -1;
            if (V == 2) {
                if ((r + l) % ri == 0) {
                    if (br > 0xFFFF) report_error(a.err, d.s + r + l, SDB_LIMIT_EXCEEDED);  // block_v2.rs:195
                    q = (int)((r + l) / ri);
                }
            } else {
                q = (int)(r + l);  // `as u16` (block.rs:163)
            }
            if (q >= 0) {
                if (tr_lds) {
                    tr[2 * q] = (uint8_t)(br >> 8);
                    tr[2 * q + 1] = (uint8_t)br;
                } else {
                    gblk[D + 2 * q] = (uint8_t)(br >> 8);
                    gblk[D + 2 * q + 1] = (uint8_t)br;
                }
            }
        }
        wave_sync();
        if (l < 16) ((lu32 *)(img - kStageGuard))[l] = 0;  // the zero lead-in of the right-aligned segments
        if (r == 0 && l == 0) ((lu32 *)img)[0] = ~((const lu32 *)img)[0];  // crc32fast's init, folded in
        wave_sync();
        crc = crc_shift_bytes(crc, Lp) ^ wave_crc_image_ra(img, Lp) ^ 0xFFFFFFFFu;
        uint8_t *gp = gblk + base;
        const uint32_t nfull = Lp >> 4;
        for (uint32_t cc = l; cc < nfull; cc += 64) {
            u32x4 v = ((const lu128 *)img)[cc];
            if (cc == 0 && r == 0) v.x = ~v.x;
            __builtin_memcpy(gp + 16 * cc, &v, 16);
        }
        if (l < (Lp & 15)) {
            const uint32_t x = (nfull << 4) + l;
            gp[x] = (r == 0 && x < 4) ? (uint8_t)~img[x] : img[x];
        }
        pu += (uint32_t)__popcll(__ballot(prow && kind == SDB_KIND_VALUE));
        de += (uint32_t)__popcll(__ballot(prow && kind == SDB_KIND_TOMBSTONE));
        me += (uint32_t)__popcll(__ballot(prow && kind == SDB_KIND_MERGE));
        base += Lp;
        r += c;
        wave_sync();
    }
    if (base != D && l == 0) report_error(a.err, d.s, SDB_DEVICE_ERROR);  // internal consistency
    if (tr_lds) {
        if (l == 0) {
            tr[2 * noffs] = (uint8_t)(noffs >> 8);
            tr[2 * noffs + 1] = (uint8_t)noffs;
        }
        wave_sync();
        const uint8_t v = l < Tl ? tr[l] : 0;
        if (l < 16) ((lu32 *)(img - kStageGuard))[l] = 0;
        img[l] = v;
        wave_sync();
        crc = crc_shift_bytes(crc, Tl) ^ wave_crc_image_ra(img, Tl) ^ 0xFFFFFFFFu;
        if (l < Tl) gblk[D + l] = v;
    } else {
        if (l == 0) {
            gblk[D + 2 * noffs] = (uint8_t)(noffs >> 8);
            gblk[D + 2 * noffs + 1] = (uint8_t)noffs;
        }
        __threadfence_block();
        wave_sync();
    }
    // a long trailer [D, Lc) read back through the image in <= 4 KiB windows
    for (uint32_t t = tr_lds ? Lc : D; t < Lc; t += 4096) {
        const uint32_t w = Lc - t < 4096 ? Lc - t : 4096;
        for (uint32_t q = l; q < w; q += 64) img[q] = gblk[t + q];
        if (l < 16) ((lu32 *)(img - kStageGuard))[l] = 0;
        for (uint32_t q = w + l; q < ((w + 63) & ~63u); q += 64) img[q] = 0;
        wave_sync();
        crc = crc_shift_bytes(crc, w) ^ wave_crc_image_ra(img, w) ^ 0xFFFFFFFFu;
        wave_sync();
    }
    crc ^= 0xFFFFFFFFu;
    if (l == 0) {
        gblk[Lc] = (uint8_t)(crc >> 24);
        gblk[Lc + 1] = (uint8_t)(crc >> 16);
        gblk[Lc + 2] = (uint8_t)(crc >> 8);
        gblk[Lc + 3] = (uint8_t)crc;
        a.out_block_stats[3 * (uint64_t)blk] = (uint16_t)pu;
        a.out_block_stats[3 * (uint64_t)blk + 1] = (uint16_t)de;
        a.out_block_stats[3 * (uint64_t)blk + 2] = (uint16_t)me;
        a.out_index_key_len[blk] = ik;
    }
    wave_sync();
}

// One wave per block, blocks strided over the grid's waves; each wave runs a two-stage software
// pipeline: while block i is assembled, CRC'd and stored from LDS, block i + 1's granules and row
// metadata are in flight into registers, and block i + 2's descriptor behind them.
template <int V>
SDB_DEV void emit_slow_blocks(const EncodeArgs &a, uint8_t *scratch, const uint32_t (*s_crc)[256]);

// SstStats / status of the encode, written by the last k_emit workgroup to finish.
SDB_DEV void finish_summary(const EncodeArgs &a) {
    sdb_sst_summary *s = a.summary;
    const unsigned long long e = atomicOr(a.err, 0ull);  // device-scope read of the error word
    s->max_block_entries = *a.wmax;
    uint64_t bl = a.bloom_len;
    if (a.bloom_len_dev) {
        bl = *a.bloom_len_dev;
        if (bl == ~0ull) {  // a prefix longer than its key (the reference asserts) or a short bitmap
            bl = 0;
            if (e == ~0ull) {
                s->status = SDB_INVALID_ARGUMENT;
                s->first_error_entry = 0;
            }
        }
    }
    s->bloom_len = bl;
    s->num_probes = a.num_probes;
    s->filter_built = a.filter_built;
    if (e != ~0ull) {
        s->status = (int32_t)(e & 0xFF);
        s->first_error_entry = e >> 8;
    }
}

// One wave per block, blocks strided over the grid's waves; each wave runs a two-stage software
// pipeline: while block i is assembled, CRC'd and stored from LDS, block i + 1's granules and row
// metadata are in flight into registers, and block i + 2's descriptor behind them.  Blocks that do
// not fit the LDS image (k_enum's slow list) are done first, one workgroup each.  The last
// workgroup to finish writes the summary.
template <int V>
__global__ __launch_bounds__(kEmitThreads, 1) void k_emit(SstSet P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#ifdef SDB_PHASE_TIMING
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), wpb = blockDim.x >> 6;
    const uint32_t gw = blockIdx.x * wpb + wave;
    (void)gw;
    const uint32_t l = (uint32_t)lane_id();
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // the set's blocks, SST after SST: lane j < count holds pre[j + 1] = blocks of SSTs <= j (an SST with
    // an earlier error, incl. capacity, emits nothing).  Kept in a VGPR, not an SGPR array: the loop's
    // scalar state must stay small (k_emit ran out of SGPRs and spilled them to VGPR lanes).
    uint32_t nbl = 0;
    if (l < P.count) {
        const EncodeArgs ai = make_args(P, l);
        if (*ai.err == ~0ull) nbl = ai.anchor_blk[ai.nchunks];
    }
    const uint32_t vpre = wave_incl_scan(nbl);
    const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)vpre, kMaxSsts - 1);
    bool run = nb > 0;
    if (lds_addr((const void *)smem) != 0) {  // crc_tab / crc_mul256_lds / crc_tree_mul assume LDS address 0
        if (threadIdx.x == 0)
            for (uint32_t i = 0; i < P.count; i++) report_error(make_args(P, i).err, 0, SDB_DEVICE_ERROR);
        run = false;
    }
    // global block g -> (SST, block of that SST); g is wave-uniform: si = #{j in [1, 8): pre[j] <= g, pre[j] < nb}
    auto locate = [&](uint32_t g, uint32_t &si, uint32_t &lb) {
        const uint64_t m = __ballot(l + 1 < kMaxSsts && vpre <= g && vpre < nb);
        si = (uint32_t)__popcll(m);
        lb = g - (si ? (uint32_t)__builtin_amdgcn_readlane((int)vpre, (int)si - 1) : 0u);
    };
    // lanes 0..13: the 14 dwords of g's desc (g clamped to the share's last block, r1 > r0: an
    // unconditional load, see emit_prefetch)
    auto desc_lanes = [&](uint32_t g, uint32_t r1) -> uint32_t {
        uint32_t si, lb;
        locate(g < r1 ? g : r1 - 1, si, lb);
        return ((const uint32_t *)make_args(P, si).desc)[14 * (uint64_t)lb + (l < 14 ? l : 13)];
    };
    if (run) {
        lu32 *crc = (lu32 *)smem;
        (void)crc;
        // schedule: workgroup b owns an equal share [r0, r1) of the set's blocks; its waves start on
        // blocks r0 + wave and then take the rest in order from an LDS ticket, so a wave that runs fast
        // takes more.  (One global ticket for all waves measured 3x slower: the atomics serialise.)
        const uint32_t r0 = (uint32_t)((uint64_t)nb * blockIdx.x / gridDim.x);
        const uint32_t r1 = (uint32_t)((uint64_t)nb * (blockIdx.x + 1) / gridDim.x);
        uint32_t blk = r0 + wave;
        const bool any = blk < r1;
        // the first block's descriptor is in flight while the CRC tables are copied, its values and
        // metadata while the workgroup does the slow blocks and sets up the ticket
        uint32_t dvc = any ? desc_lanes(blk, r1) : 0u;
#ifdef SDB_EMIT_CRC_SLICE
        crc_tables_to_lds(crc);
#else
        crc_mfma_tables_to_lds(crc);
#endif
        EmitData pd;
        EmitMeta mc;
        bool fc = false;
        if (any) {
            uint32_t si, lb;
            locate(blk, si, lb);
            const BlockDesc d0 = desc_from_lanes(dvc);
            fc = emit_fast(d0);
            emit_prefetch_data(make_args(P, si), desc_or_empty(d0, fc), pd);
            emit_prefetch_meta(make_args(P, si), desc_or_empty(d0, fc), mc);
        }
        __syncthreads();
        for (uint32_t i = 0; i < P.count; i++) {
            const EncodeArgs ai = make_args(P, i);
            if (*ai.err == ~0ull && *ai.slow_count)
#ifdef SDB_EMIT_CRC_SLICE
                emit_slow_blocks<V>(ai, (uint8_t *)smem + kCrcLds + 16, (const uint32_t(*)[256])smem);
#else  // (the rare workgroup path reads the slicing tables from constant memory)
                emit_slow_blocks<V>(ai, (uint8_t *)smem + kCrcLds + 16, (const uint32_t(*)[256])c_crc.t);
#endif
        }
        __syncthreads();
        if (threadIdx.x == 0) *(lu32 *)(smem + kCrcLds) = blockDim.x >> 6;  // block ticket (first blocks: r0 + wave)
        __syncthreads();
        lu8 *wbase = (lu8 *)smem + kCrcLds + 16 + wave * kEmitWaveLds;
        lu8 *img = wbase + kStageGuard;
        lu8 *kst = img + kImgCap + 16;
        lSpanCopy *rtab = (lSpanCopy *)(kst + kKeyStageCap);
        lu32 *ticket = (lu32 *)(smem + kCrcLds);
        auto take = [&]() -> uint32_t {
            uint32_t t = 0;
            if (l == 0) t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return r0 + (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
        };
        if (any) {
            // Software pipeline, one block deep: while block `blk` is assembled (its data pc landed), the
            // next block's data and the descriptor of the one after it are in flight.  Every iteration
            // issues exactly the same memory instructions (unconditional loads, range-checked stores, the
            // last iteration's prefetch wasted), and the state entering the loop has nothing in flight, so
            // the compiler's only vmcnt waits are the end-of-iteration hand-overs (pn -> pc, dv2 -> dvn),
            // which leave this block's stores in flight.
            uint32_t nblk = take();
            uint32_t dvn = desc_lanes(nblk, r1);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            while (true) {
                // block blk's data landed (the hand-over wait at the end of the previous iteration): stage
                // it, then its registers take the next block's data
                emit_stage(desc_or_empty(desc_from_lanes(dvc), fc), pd, img, kst);
                const bool more = nblk < r1;
                uint32_t si, lb;
                locate(more ? nblk : r1 - 1, si, lb);
                const BlockDesc dn0 = desc_from_lanes(dvn);
                const bool fn = more && emit_fast(dn0);
                const BlockDesc dn = desc_or_empty(dn0, fn);
                emit_prefetch_data(make_args(P, si), dn, pd);
                EmitMeta mn;
                emit_prefetch_meta(make_args(P, si), dn, mn);
                const uint32_t n2 = take();
                const uint32_t dv2 = desc_lanes(n2, r1);
                uint32_t csi, clb;
                locate(blk, csi, clb);  // others: k_emit_big, slow path (emitted empty, stores dropped)
                emit_block<V>(make_args(P, csi), clb, desc_or_empty(desc_from_lanes(dvc), fc), fc, mc, img, kst, rtab, crc, ph);
                if (!more) break;
                blk = nblk;
                nblk = n2;
                dvc = dvn;
                dvn = dv2;
                mc = mn;
                fc = fn;
            }
        }
    }
#ifdef SDB_PHASE_TIMING
    if (lane_id() == 0 && gw < 8192)
        for (int i = 0; i < 8; i++) g_wave_phase[gw][i] = ph[i];
    const uint64_t rt1 = __builtin_amdgcn_s_memrealtime(), mt1 = __builtin_amdgcn_s_memtime();
    if (lane_id() == 0 && gw < 8192) {
        g_wave_rt[gw][0] = rt0;
        g_wave_rt[gw][1] = rt1;
        g_wave_rt[gw][2] = mt0;
        g_wave_rt[gw][3] = mt1;
    }
#endif
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&make_args(P, 0).done[0], 1u) == gridDim.x - 1) {
            __threadfence();
            for (uint32_t i = 0; i < P.count; i++) finish_summary(make_args(P, i));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// K6: slow path for blocks that do not fit the LDS image: assemble straight into HBM.
// ------------------------------------------------------------------------------------------------
template <int V>
SDB_DEV void emit_slow_blocks(const EncodeArgs &a, uint8_t *scratch, const uint32_t (*s_crc)[256]) {
    // LDS scratch (the wave images, unused until the fast loop): window, row sizes, row offsets
    uint8_t *s_win = scratch;  // 4096 + 64, window at +16
    uint64_t *s_size = (uint64_t *)(scratch + 8192);
    uint64_t *s_off = (uint64_t *)(scratch + 8192 + 8 * kEmitThreads);
    const uint32_t nslow = *a.slow_count;
    for (uint32_t it = blockIdx.x; it < nslow; it += gridDim.x) {
        const uint32_t blk = a.slow_list[it];
        const uint64_t b = a.out_block_first[blk];
        const uint64_t e = a.next[b];
        const uint64_t off = a.out_block_off[blk];
        const uint32_t ne = (uint32_t)(e - b);
        uint8_t *dst = a.out_data + off;
        const uint32_t ri = a.restart_interval;
        const uint64_t fko = a.key_off[b];
        const uint32_t fkl = (uint32_t)(a.key_off[b + 1] - fko);
        uint64_t D = 0;
        for (uint32_t i0 = 0; i0 < ne; i0 += blockDim.x) {
            uint32_t i = i0 + threadIdx.x;
            // each thread writes its own row; row offsets need a prefix sum -> do it serially per round
            RowInfo r;
            uint64_t seq = 0;
            int64_t ets = 0, cts = 0;
            if (i < ne) {
                uint64_t j = b + i;
                uint64_t ko = a.key_off[j];
                uint32_t klen = (uint32_t)(a.key_off[j + 1] - ko);
                uint8_t kd = a.kind ? a.kind[j] : 0;
                uint8_t m = a.ts_mask ? a.ts_mask[j] : 0;
                uint32_t vlen = kd == SDB_KIND_TOMBSTONE ? 0 : (uint32_t)(a.val_off[j + 1] - a.val_off[j]);
                uint32_t shared;
                if (V == 2) shared = (i % ri == 0) ? 0 : a.lcp[j];
                else shared = (i == 0) ? 0 : lcp_bytes(a.key_bytes + fko, fkl, a.key_bytes + ko, klen);
                r.shared = shared;
                r.suf = klen - shared;
                r.vlen = vlen;
                r.key_src = ko + shared;
                r.val_src = a.val_off[j];
                r.flags = (uint8_t)((kd == SDB_KIND_MERGE ? SDB_FLAG_MERGE_OPERAND : 0) |
                                    (kd == SDB_KIND_TOMBSTONE ? SDB_FLAG_TOMBSTONE : 0) |
                                    ((m & SDB_TS_EXPIRE) ? SDB_FLAG_HAS_EXPIRE_TS : 0) |
                                    ((m & SDB_TS_CREATE) ? SDB_FLAG_HAS_CREATE_TS : 0));
                const uint32_t ts8 = 8u * (((m & SDB_TS_CREATE) != 0) + ((m & SDB_TS_EXPIRE) != 0));
                if (V == 2) r.size = varint_len(shared) + varint_len(r.suf) + varint_len(vlen) + r.suf + vlen + 9 + ts8;
                else r.size = 4 + r.suf + 9 + ts8 + (kd == SDB_KIND_TOMBSTONE ? 0 : 4 + vlen);
                seq = a.seq ? a.seq[j] : 0;
                ets = (m & SDB_TS_EXPIRE) ? a.expire_ts[j] : 0;
                cts = (m & SDB_TS_CREATE) ? a.create_ts[j] : 0;
                s_size[threadIdx.x] = r.size;
            } else {
                s_size[threadIdx.x] = 0;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                uint64_t c = D;
                for (uint32_t q = 0; q < blockDim.x; q++) {
                    s_off[q] = c;
                    c += s_size[q];
                }
            }
            __syncthreads();
            if (i < ne) {
                uint64_t ro = s_off[threadIdx.x];
                r.row_off = (uint32_t)ro;
                uint8_t *row = dst + ro;
                uint32_t h;
                write_row_small<V>(row, r, seq, ets, cts, &h);
                for (uint32_t q = 0; q < r.suf; q++) row[h + q] = a.key_bytes[r.key_src + q];
                uint32_t voff = (V == 2) ? h + r.suf : (r.size - r.vlen);
                for (uint32_t q = 0; q < r.vlen; q++) row[voff + q] = a.val_bytes[r.val_src + q];
                // offsets
                if (V == 2) {
                    if (i % ri == 0) {
                        if (ro > 0xFFFF) report_error(a.err, b + i, SDB_LIMIT_EXCEEDED);
                        // placed after all rows: remember in s_off reuse below
                    }
                }
            }
            __syncthreads();
            // offsets table entries for this round are written after D is known: store row offsets
            // temporarily in the workspace `lcp` is still needed, so stash into row_scratch (per entry)
            if (i < ne) a.row_scratch[b + i] = (uint32_t)s_off[threadIdx.x];
            D = s_off[blockDim.x - 1] + s_size[blockDim.x - 1];
            __syncthreads();
        }
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) {  // BlockStats + compute_index_key for this block
            uint32_t pu = 0, de = 0, me = 0;
            for (uint64_t j = b; j < e; j++) {
                uint8_t kd = a.kind ? a.kind[j] : 0;
                pu += kd == SDB_KIND_VALUE;
                de += kd == SDB_KIND_TOMBSTONE;
                me += kd == SDB_KIND_MERGE;
            }
            a.out_block_stats[3 * (uint64_t)blk] = (uint16_t)pu;
            a.out_block_stats[3 * (uint64_t)blk + 1] = (uint16_t)de;
            a.out_block_stats[3 * (uint64_t)blk + 2] = (uint16_t)me;
            uint32_t ik = 0;
            if (b > 0 && !a.wal) {
                uint64_t fl = a.key_off[b + 1] - a.key_off[b];
                uint64_t pl = a.key_off[b] - a.key_off[b - 1];
                uint32_t lc = a.lcp[b];
                ik = (lc == pl && pl == fl) ? (uint32_t)fl : lc + 1;
            }
            a.out_index_key_len[blk] = ik;
        }
        uint32_t noffs = (V == 2) ? (ne + ri - 1) / ri : ne;
        for (uint32_t q = threadIdx.x; q < noffs; q += blockDim.x) {
            uint32_t ro = a.row_scratch[b + (V == 2 ? (uint64_t)q * ri : q)];
            dst[D + 2 * q] = (uint8_t)(ro >> 8);
            dst[D + 2 * q + 1] = (uint8_t)ro;
        }
        if (threadIdx.x == 0) {
            dst[D + 2 * noffs] = (uint8_t)(noffs >> 8);
            dst[D + 2 * noffs + 1] = (uint8_t)noffs;
        }
        __threadfence();
        __syncthreads();
        // CRC over [dst, dst + Lc) with 4 KiB right-aligned windows staged through LDS by wave 0
        const uint64_t Lc = D + 2 * (uint64_t)noffs + 2;
        if (threadIdx.x < 64) {
            uint64_t nwin = (Lc + 4095) >> 12;
            uint64_t first = Lc - ((nwin - 1) << 12);
            uint32_t acc = 0;
            for (uint64_t w = 0; w < nwin; w++) {
                uint64_t wbeg = (w == 0) ? 0 : first + ((w - 1) << 12);
                uint32_t wlen = (uint32_t)((w == 0) ? first : 4096);
                // crc32fast's 0xFFFFFFFF init = inverting message bytes [0, 4), which straddle the
                // first two windows when the first holds fewer than 4 bytes (V1 blocks of
                // block_size + 1 or + 2 bytes: the new entry's offset is not counted, block.rs:117-123)
                for (uint32_t q = threadIdx.x; q < wlen; q += 64)
                    s_win[16 + q] = dst[wbeg + q] ^ (wbeg + q < 4 ? 0xFF : 0);
                wave_sync();
                uint32_t raw = wave_crc_raw_lds(s_win + 16, wlen, (const uint32_t(*)[256])s_crc, false);
                // R(A || B) = R(A) * x^(8|B|) + R(B); every window after the first is 4096 bytes
                acc = (w == 0) ? raw : (gf_mul(c_shift.window, acc) ^ raw);
                wave_sync();
            }
            uint32_t crc = acc ^ 0xFFFFFFFFu;
            if (threadIdx.x == 0) {
                dst[Lc] = (uint8_t)(crc >> 24);
                dst[Lc + 1] = (uint8_t)(crc >> 16);
                dst[Lc + 2] = (uint8_t)(crc >> 8);
                dst[Lc + 3] = (uint8_t)crc;
            }
        }
        __syncthreads();
    }
}

template __global__ void k_emit<1>(SstSet);
template __global__ void k_emit<2>(SstSet);

// The piece path (emit_big) in a launch of its own, before k_emit (whose last workgroup writes the
// summaries, so it sees this kernel's errors): inlined into k_emit it cost the fast path its registers.
// Waves take the set's big blocks round-robin; a set without any returns before the table copy.
template <int V>
__global__ __launch_bounds__(kEmitThreads, 1) void k_emit_big(SstSet P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t pre[kMaxSsts + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t i = 0; i < kMaxSsts; i++) {
        uint32_t nb = 0;
        if (i < P.count) {
            const EncodeArgs ai = make_args(P, i);
            if (*ai.err == ~0ull) nb = *ai.big_count;
        }
        pre[i + 1] = pre[i] + nb;
    }
    const uint32_t total = pre[kMaxSsts];
    if (!total || lds_addr((const void *)smem) != 0) return;
    crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), wpb = blockDim.x >> 6;
    lu8 *img = (lu8 *)smem + kCrcLds + 16 + wave * kEmitWaveLds + kStageGuard;
    lu8 *kst = img + kImgCap + 16;
    lSpanCopy *rtab = (lSpanCopy *)(kst + kKeyStageCap);
    for (uint32_t g = blockIdx.x * wpb + wave; g < total; g += gridDim.x * wpb) {
        uint32_t si = 0, base = 0;
#pragma unroll
        for (uint32_t j = 1; j < kMaxSsts; j++)
            if (g >= pre[j] && pre[j] < total) {
                si = j;
                base = pre[j];
            }
        const EncodeArgs a = make_args(P, si);
        const uint32_t blk = a.big_list[g - base];
        emit_big<V>(a, blk, a.desc[blk], img, kst, rtab);
    }
}
template __global__ void k_emit_big<1>(SstSet);
template __global__ void k_emit_big<2>(SstSet);

// ------------------------------------------------------------------------------------------------
// Launcher
// ------------------------------------------------------------------------------------------------
__global__ void k_init_summary(EncodeArgs a) {
    if (threadIdx.x == 0) {
        sdb_sst_summary *s = a.summary;
        s->data_len = 0;
        s->num_blocks = 0;
        s->num_entries = a.n;
        s->raw_key_size = 0;
        s->raw_val_size = 0;
        s->num_puts = s->num_deletes = s->num_merges = 0;
        s->bloom_len = 0;
        s->num_probes = 0;
        s->filter_built = 0;
        s->status = 0;
        s->max_block_entries = 0;
        s->first_error_entry = ~0ull;
        *a.err = ~0ull;
        *a.wmax = 0;
        *a.slow_count = 0;
        *a.big_count = 0;
        if (a.n == 0 && a.block_cap + 1 > 0) {  // empty SST: BlockMeta list is empty, offsets = [0]
            a.out_block_off[0] = 0;
            a.out_block_first[0] = 0;
        }
    }
}

__global__ void k_finish_summary(EncodeArgs a, uint64_t bloom_len, uint32_t num_probes, uint32_t built) {
    if (threadIdx.x == 0) {
        sdb_sst_summary *s = a.summary;
        unsigned long long e = *a.err;
        s->max_block_entries = *a.wmax;
        s->bloom_len = bloom_len;
        s->num_probes = num_probes;
        s->filter_built = built;
        if (e != ~0ull) {
            s->status = (int32_t)(e & 0xFF);
            s->first_error_entry = e >> 8;
        }
    }
}

#ifdef SDB_PHASE_TIMING
extern "C" int sdb_diag_wave_phase(uint64_t *out, int nwaves) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_phase), sizeof(uint64_t) * 8 * nwaves) == hipSuccess ? 0 : -1;
}
extern "C" int sdb_diag_wave_rt(uint64_t *out, int nwaves) {
#ifdef SDB_PHASE_TIMING
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_rt), sizeof(uint64_t) * 4 * nwaves) == hipSuccess ? 0 : -1;
#else
    return -1;
#endif
}
extern "C" int sdb_diag_enum_phase(uint64_t *out, int nblocks) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_enum), sizeof(uint64_t) * 8 * nblocks) == hipSuccess ? 0 : -1;
}
extern "C" int sdb_diag_phase_times(uint64_t *out, int nblocks) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(uint64_t) * 8 * nblocks) == hipSuccess ? 0 : -1;
}
#endif

static int g_cus = 0;
static uint32_t g_emit_threads = kEmitThreads, g_emit_wg_per_cu = kEmitWgPerCu;
static std::once_flag g_attrs_once;
static uint32_t g_emit_grid = 0;  // SDB_EMIT_GRID: an absolute k_emit grid (diagnostics)
constexpr int kMaxDevices = 64;
static std::atomic<uint32_t> g_builders[kMaxDevices];  // sdb_set_concurrent_builders, per device (0: 1)
static int current_device() {
    int dev = 0;
    return hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDevices ? dev : 0;
}
// k_emit is persistent (one workgroup per CU, most of its LDS): with B builders in flight it takes 1/B of
// the CUs, so another builder's latency-bound segmentation runs beside it instead of queueing behind it
// (two builders at 128 of 256 CUs: +7 % over one builder on the whole chip)
static uint32_t emit_grid() {
    if (g_emit_grid) return g_emit_grid;
    const uint32_t full = (uint32_t)(g_cus > 0 ? g_emit_wg_per_cu * g_cus : 512);
    const uint32_t b = g_builders[current_device()].load(std::memory_order_relaxed);
    return b > 1 ? (full / b ? full / b : 1u) : full;
}
static uint32_t emit_lds() { return kCrcLds + 16 + (g_emit_threads / 64) * kEmitWaveLds; }
static void set_lds_attrs() {
    std::call_once(g_attrs_once, [] {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
        // tuning knobs (diagnostics): emit workgroup size and workgroups per CU
        if (const char *e = getenv("SDB_EMIT_THREADS")) {
            uint32_t t = (uint32_t)atoi(e);
            if (t >= 64 && t <= kEmitThreads && t % 64 == 0) g_emit_threads = t;
        }
        if (const char *e = getenv("SDB_EMIT_GRID")) {
            const int t = atoi(e);
            if (t >= 1 && t <= 4096) g_emit_grid = (uint32_t)t;
        }
        if (const char *e = getenv("SDB_EMIT_WG_PER_CU")) {
            uint32_t t = (uint32_t)atoi(e);
            if (t >= 1 && t <= 32) g_emit_wg_per_cu = t;
        }
        (void)hipFuncSetAttribute((const void *)k_emit<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds);
        (void)hipFuncSetAttribute((const void *)k_emit<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds);
        (void)hipFuncSetAttribute((const void *)k_emit_big<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds);
        (void)hipFuncSetAttribute((const void *)k_emit_big<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds);
        (void)hipFuncSetAttribute((const void *)k_enum, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEnumLds);
        (void)hipFuncSetAttribute((const void *)k_group, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGroupLds);
        (void)hipFuncSetAttribute((const void *)k_anchor, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAnchorLds);
        (void)hipFuncSetAttribute((const void *)k_seg, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        (void)hipFuncSetAttribute((const void *)k_facts, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLds);
        (void)hipGetLastError();  // an unsupported attribute value must not poison the next launch status
    });
}

// ------------------------------------------------------------------------------------------------
// Bloom (fused with the encode): k_facts bins each chunk's probes into (tile, slice) slots, and
// workgroups of k_seg past its chunks OR one slice's slots into LDS and write the bitmap slice
// (sdb_bloom.h).
// ------------------------------------------------------------------------------------------------
static_assert(kChunk == kFactsEntries && kFactsThreads == kBinThreads, "bloom tiles are k_facts' chunks of kChunk keys");

hipError_t launch_encode_set(const SstSet &P, size_t bin_lds, size_t fill_lds, hipStream_t st) {
    set_lds_attrs();
    if (!P.count) return hipSuccess;
    // every kernel on the caller's stream, in dependency order: the set is large enough to fill the
    // chip at each step, and one stream keeps the sequence capturable into a HIP graph
    stage_mark(st, kStFacts, true);
    hipLaunchKernelGGL(k_facts, dim3(P.max_facts, P.count), dim3(kFactsThreads), P.max_tiles ? bin_lds : 0, st, P);
    stage_mark(st, kStFacts, false);
    stage_mark(st, kStSeg, true);
    // k_seg also fills the fused bloom's slices (workgroups past the chunks)
    const size_t seg_lds = kSegLds > fill_lds ? kSegLds : fill_lds;
    hipLaunchKernelGGL(k_seg, dim3(P.max_chunks + P.max_slices, P.count), dim3(kSegThreads), seg_lds, st, P);
    stage_mark(st, kStSeg, false);
    // the chain: every chunk's anchor (one workgroup per SST), then each chunk's blocks
    stage_mark(st, kStAnchor, true);
    hipLaunchKernelGGL(k_anchor, dim3(1, P.count), dim3(kAnchorThreads), kAnchorLds, st, P);
    stage_mark(st, kStAnchor, false);
    stage_mark(st, kStBlocks, true);
    hipLaunchKernelGGL(k_blocks, dim3(P.max_chunks, P.count), dim3(kBlkThreads), 0, st, P);
    stage_mark(st, kStBlocks, false);
    stage_mark(st, kStEmitBig, true);
    // blocks over one wave image: every block at SstBlockSize 8 - 64 KiB, only blocks of > 64 tiny rows
    // at 4 KiB and below (a small grid: a full grid of 137 KB workgroups that find nothing to do costs
    // ~7 us per set)
    const uint32_t big_grid = P.block_size > 4096 ? emit_grid() : (emit_grid() < 32 ? emit_grid() : 32);
    if (P.version == 2) hipLaunchKernelGGL(k_emit_big<2>, dim3(big_grid), dim3(g_emit_threads), emit_lds(), st, P);
    else hipLaunchKernelGGL(k_emit_big<1>, dim3(big_grid), dim3(g_emit_threads), emit_lds(), st, P);
    stage_mark(st, kStEmitBig, false);
    stage_mark(st, kStEmit, true);  // k_emit alone (the kernel bench.py's roofline entry times)
    if (P.version == 2) hipLaunchKernelGGL(k_emit<2>, dim3(emit_grid()), dim3(g_emit_threads), emit_lds(), st, P);
    else hipLaunchKernelGGL(k_emit<1>, dim3(emit_grid()), dim3(g_emit_threads), emit_lds(), st, P);
    stage_mark(st, kStEmit, false);
    return hipGetLastError();
}

// The block chain alone (k_facts -> k_seg -> k_group): per-entry next() / block bytes, the chunk and
// group transfer tables and the walk mode, for the compactor's SST cuts (sdb_compact.hip).  The slot
// builds no filter.
hipError_t launch_encode_prep(const SstSet &P, hipStream_t st) {
    set_lds_attrs();
    if (!P.count) return hipSuccess;
    hipLaunchKernelGGL(k_facts, dim3(P.max_facts, P.count), dim3(kFactsThreads), 0, st, P);
    hipLaunchKernelGGL(k_seg, dim3(P.max_chunks, P.count), dim3(kSegThreads), kSegLds, st, P);
    hipLaunchKernelGGL(k_group, dim3(P.max_groups, P.count), dim3(kGroupThreads), kGroupLds, st, P);
    return hipGetLastError();
}

// An empty SST (no entries): summary only, BlockMeta offsets = [0].
hipError_t launch_encode_empty(EncodeArgs a, hipStream_t st) {
    hipLaunchKernelGGL(k_init_summary, dim3(1), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_finish_summary, dim3(1), dim3(64), 0, st, a, a.bloom_len, a.num_probes, a.filter_built);
    return hipGetLastError();
}

}  // namespace sdb

extern "C" sdb_status sdb_set_concurrent_builders(uint32_t builders) {
    if (builders == 0) return SDB_INVALID_ARGUMENT;
    sdb::g_builders[sdb::current_device()].store(builders, std::memory_order_relaxed);
    return SDB_OK;
}
