// sdb_decode.hip — batched SST block decode for gfx950.
//
// Replaces SsTableFormat::read_blocks -> decode_block -> validate_checksum -> Block::decode
// (slatedb/src/format/sst.rs:938-1038, format/block.rs:28-46) followed by draining
// DataBlockIterator ascending (block_iterator.rs:54-267, block_iterator_v2.rs:33-113,235-267) into
// columnar RowEntry output (the SstFile::read_block contract, sst_reader.rs:287-309).
//
// D1 count   one wave per block: stage the block into LDS with 16-byte loads, CRC32 check
//            (same wave CRC as the encoder), parse the trailer and every row (V2: one lane per
//            restart region; V1: one lane per entry offset) -> entries and restored-key bytes.
// D2 scan    exclusive scans over blocks (tile sums -> tile scan -> apply).
// D3 emit    one wave per block: parse again and write keys (restored against the previous key),
//            value references into `blocks`, seq, flags and timestamps.
#include <mutex>
#include <type_traits>

#include "sdb_decode.h"
#include "sdb_crc.h"
#include "sdb_crc_mfma.h"
#include "sdb_device.h"

namespace sdb {

#ifdef SDB_PHASE_TIMING
__device__ uint64_t g_dec_phase[2][8192][4];  // [count / emit][wave][phase] s_memtime ticks
#define DEC_T(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define DEC_ACC(pass, ph, dt) \
    do { if (lane_id() == 0 && gwave < 8192) g_dec_phase[pass][gwave][ph] += (dt); } while (0)
#else
#define DEC_T(var) do { } while (0)
#define DEC_ACC(pass, ph, dt) do { } while (0)
#endif
// geometry of the count and emit passes (diagnostic knobs): threads per workgroup, workgroups per CU
#ifndef SDB_CNT_THREADS
#define SDB_CNT_THREADS 1024
#endif
#ifndef SDB_CNT_WG
#define SDB_CNT_WG 1
#endif
#ifndef SDB_EM_THREADS
#define SDB_EM_THREADS 1024
#endif
#ifndef SDB_EM_WG
#define SDB_EM_WG 1
#endif
constexpr uint32_t kCntThreads = SDB_CNT_THREADS, kCntWg = SDB_CNT_WG, kEmThreads = SDB_EM_THREADS, kEmWg = SDB_EM_WG;
constexpr uint32_t kCntEu = (kCntThreads / 64 * kCntWg + 3) / 4, kEmEu = (kEmThreads / 64 * kEmWg + 3) / 4;  // waves per SIMD
constexpr uint32_t kDecImg = 4096 + 32;                  // fast path: staged block image per wave
constexpr uint32_t kDecKeys = 2048;                      // fast path: restored keys of one block
constexpr uint32_t kDecGuard = 64;                       // zero lead-in of the right-aligned CRC segments
constexpr uint32_t kDecWaveLds = kDecGuard + kDecImg + kDecKeys;
// the checksum of a staged block (crc_staged_ok: the count pass, fail-fast emit): slicing-by-8 (36 KiB
// of tables), or (SDB_DEC_CRC_MFMA) on the matrix cores (sdb_crc_mfma.h: weights + tree tables, 56 KiB
// at LDS 0), which measured slower on configs[2] (0.947 vs 0.898 ms)
#ifndef SDB_DEC_CRC_MFMA
#define SDB_DEC_CRC_SLICE
#endif
#ifdef SDB_DEC_CRC_SLICE
constexpr uint32_t kDecTabLds = kCrcTablesLds;
#else
constexpr uint32_t kDecTabLds = kCrcMfmaLds;
#endif
SDB_DEV void dec_crc_tables_to_lds(lu32 *at) {
#ifdef SDB_DEC_CRC_SLICE
    crc_tables_to_lds(at);
#else
    crc_mfma_tables_to_lds(at);
#endif
}
constexpr uint32_t kDecLds = kDecTabLds + (kEmThreads / 64) * kDecWaveLds;  // emit: tables (fail-fast CRC), waves
constexpr uint32_t kDecCap = kDecWaveLds - kDecGuard;
// count pass: the CRC tables, the bank-replicated byte table (sdb_crc.h), then per wave a guard + image
constexpr uint32_t kCntWaveLds = kDecGuard + kDecImg;
constexpr uint32_t kCntLds = kDecTabLds + (kCntThreads / 64) * kCntWaveLds;
static_assert(kCntLds <= 160 * 1024, "count pass LDS");
constexpr uint32_t kRowTmp = kDecKeys - 256;  // emit: row positions of the lane-per-row path (4 x 32 u16) in kbuf
typedef __attribute__((address_space(3))) uint16_t lu16;  // other blocks: generic staging per wave; larger ones parse from HBM

template <typename P>
SDB_DEV uint64_t rd_be(P p, int nb) {
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
    return v;
}

// Parse one varint (decode_varint, utils.rs:622-634) from d[*pos] (bounded by end).
template <typename P>
SDB_DEV bool rd_varint(P d, uint32_t end, uint32_t *pos, uint32_t *v) {
    uint32_t r = 0;
    int sh = 0;
    for (;;) {
        if (*pos >= end || sh > 28) return false;
        uint8_t b = d[(*pos)++];
        r |= (uint32_t)(b & 0x7F) << sh;
        if (!(b & 0x80)) break;
        sh += 7;
    }
    *v = r;
    return true;
}

// Block k is blocks[block_off[k] .. end): contiguous blocks end where the next begins; scattered
// blocks (sdb_decode_blocks_at: many read_blocks ranges in one arena) carry their own ends.
SDB_DEV uint64_t block_end_of(const DecodeArgs &a, uint64_t k) { return a.block_end ? a.block_end[k] : a.block_off[k + 1]; }

SDB_DEV bool flags_ok(uint8_t f) {  // decode_flags (row_codec_v2.rs:234-249)
    return !(f & ~0x0Fu) && !((f & SDB_FLAG_TOMBSTONE) && (f & SDB_FLAG_MERGE_OPERAND));
}

struct RowV2 {
    uint32_t shared, unshared, vlen, suf_pos, val_pos, next;
    uint64_t seq;
    int64_t ets, cts;
    uint8_t flags;
};

// SstRowCodecV2::decode (row_codec_v2.rs:172-220).  Returns 0 or an sdb_status.
template <typename P>
SDB_DEV int parse_v2(P d, uint32_t end, uint32_t pos, RowV2 *r) {
    if (!rd_varint(d, end, &pos, &r->shared) || !rd_varint(d, end, &pos, &r->unshared) ||
        !rd_varint(d, end, &pos, &r->vlen))
        return SDB_CORRUPT_BLOCK;
    if ((uint64_t)pos + r->unshared + r->vlen + 9 > end) return SDB_CORRUPT_BLOCK;
    r->suf_pos = pos;
    pos += r->unshared;
    r->val_pos = pos;
    pos += r->vlen;
    r->seq = rd_be(d + pos, 8);
    pos += 8;
    uint8_t f = d[pos++];
    if (!flags_ok(f)) return SDB_INVALID_ROW_FLAGS;
    uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > end) return SDB_CORRUPT_BLOCK;
    r->ets = 0;
    r->cts = 0;
    if (f & SDB_FLAG_HAS_EXPIRE_TS) {
        r->ets = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    if (f & SDB_FLAG_HAS_CREATE_TS) {
        r->cts = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    r->flags = f;
    r->next = pos;
    return 0;
}

// The same decode for rows staged in LDS: the header and the trailer are each read as one unaligned
// 16-byte window (five aligned dwords + v_alignbyte, all in flight together) instead of byte by byte,
// and single-byte varints (every length < 128) decode from the window in registers.
SDB_DEV void lds_read16(const lu8 *p, uint32_t (&w)[4]) {
    const uint32_t addr = lds_addr((const void *)p), sh = addr & 3;
    const lu32 *d = (const lu32 *)(uintptr_t)(addr & ~3u);
    const uint32_t x0 = d[0], x1 = d[1], x2 = d[2], x3 = d[3], x4 = d[4];
    w[0] = __builtin_amdgcn_alignbyte(x1, x0, sh);
    w[1] = __builtin_amdgcn_alignbyte(x2, x1, sh);
    w[2] = __builtin_amdgcn_alignbyte(x3, x2, sh);
    w[3] = __builtin_amdgcn_alignbyte(x4, x3, sh);
}
SDB_DEV uint64_t be64_at(uint32_t lo, uint32_t hi) { return __builtin_bswap64((uint64_t)lo | ((uint64_t)hi << 32)); }

SDB_DEV int parse_v2(const lu8 *d, uint32_t end, uint32_t pos, RowV2 *r) {
    uint32_t w[4];
    lds_read16(d + pos, w);
    if ((w[0] & 0x808080u) == 0 && pos + 3 <= end) {
        r->shared = w[0] & 0x7F;
        r->unshared = (w[0] >> 8) & 0x7F;
        r->vlen = (w[0] >> 16) & 0x7F;
        pos += 3;
    } else if (!rd_varint(d, end, &pos, &r->shared) || !rd_varint(d, end, &pos, &r->unshared) ||
               !rd_varint(d, end, &pos, &r->vlen)) {
        return SDB_CORRUPT_BLOCK;
    }
    if ((uint64_t)pos + r->unshared + r->vlen + 9 > end) return SDB_CORRUPT_BLOCK;
    r->suf_pos = pos;
    pos += r->unshared;
    r->val_pos = pos;
    pos += r->vlen;
    uint32_t x[4];
    lds_read16(d + pos, x);  // seq (8), flags (1), the first 7 bytes of the timestamps
    r->seq = be64_at(x[0], x[1]);
    const uint8_t f = (uint8_t)x[2];
    pos += 9;
    if (!flags_ok(f)) return SDB_INVALID_ROW_FLAGS;
    const uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > end) return SDB_CORRUPT_BLOCK;
    r->ets = 0;
    r->cts = 0;
    if (need) {
        uint32_t y[4];
        lds_read16(d + pos + 7, y);  // bytes 16.. of the trailer window
        // trailer bytes 9..16 and 17..24 as little-endian dword pairs
        const uint32_t t0 = __builtin_amdgcn_alignbyte(x[3], x[2], 1), t1 = __builtin_amdgcn_alignbyte(y[0], x[3], 1);
        const uint32_t t2 = __builtin_amdgcn_alignbyte(y[1], y[0], 1), t3 = __builtin_amdgcn_alignbyte(y[2], y[1], 1);
        const int64_t first = (int64_t)be64_at(t0, t1), second = (int64_t)be64_at(t2, t3);
        if (f & SDB_FLAG_HAS_EXPIRE_TS) {
            r->ets = first;
            if (f & SDB_FLAG_HAS_CREATE_TS) r->cts = second;
        } else {
            r->cts = first;
        }
    }
    r->flags = f;
    r->next = pos + need;
    return 0;
}

// The same decode straight from HBM (blocks over one wave image): 16-byte unaligned vector loads for
// the header and the trailer instead of ~15 dependent byte loads per row.  `end` is the end of the rows;
// the block's offsets, count and CRC (>= 8 bytes) follow, so a window is read whole while it ends
// within end + 8, byte by byte otherwise.
typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));
SDB_DEV void g_read16(const uint8_t *p, uint32_t avail, uint32_t (&w)[4]) {
    if (avail >= 16) {
        const u32x4_ua v = *(const u32x4_ua *)p;
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
        return;
    }
    w[0] = w[1] = w[2] = w[3] = 0;
    for (uint32_t i = 0; i < avail && i < 16; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
}

SDB_DEV int parse_v2(const uint8_t *d, uint32_t end, uint32_t pos, RowV2 *r) {
    const uint32_t lim = end + 8;
    uint32_t w[4];
    g_read16(d + pos, pos < lim ? lim - pos : 0, w);
    if ((w[0] & 0x808080u) == 0 && pos + 3 <= end) {
        r->shared = w[0] & 0x7F;
        r->unshared = (w[0] >> 8) & 0x7F;
        r->vlen = (w[0] >> 16) & 0x7F;
        pos += 3;
    } else if (!rd_varint(d, end, &pos, &r->shared) || !rd_varint(d, end, &pos, &r->unshared) ||
               !rd_varint(d, end, &pos, &r->vlen)) {
        return SDB_CORRUPT_BLOCK;
    }
    if ((uint64_t)pos + r->unshared + r->vlen + 9 > end) return SDB_CORRUPT_BLOCK;
    r->suf_pos = pos;
    pos += r->unshared;
    r->val_pos = pos;
    pos += r->vlen;
    uint32_t x[4];
    g_read16(d + pos, pos < lim ? lim - pos : 0, x);  // seq (8), flags (1), the first 7 bytes of the timestamps
    r->seq = __builtin_bswap64((uint64_t)x[0] | ((uint64_t)x[1] << 32));
    const uint8_t f = (uint8_t)x[2];
    pos += 9;
    if (!flags_ok(f)) return SDB_INVALID_ROW_FLAGS;
    const uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > end) return SDB_CORRUPT_BLOCK;
    r->ets = 0;
    r->cts = 0;
    if (f & SDB_FLAG_HAS_EXPIRE_TS) {
        r->ets = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    if (f & SDB_FLAG_HAS_CREATE_TS) {
        r->cts = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    r->flags = f;
    r->next = pos;
    return 0;
}

struct RowV0 {
    uint32_t prefix, suf, suf_pos, vlen, val_pos;
    uint64_t seq;
    int64_t ets, cts;
    uint8_t flags;  // as returned by the iterator (V0 tombstones drop expire_ts, row.rs:223-231)
};

// SstRowCodecV0::decode (row.rs:200-249).
template <typename P>
SDB_DEV int parse_v0(P d, uint32_t end, uint32_t pos, RowV0 *r) {
    if ((uint64_t)pos + 4 > end) return SDB_CORRUPT_BLOCK;
    r->prefix = (uint32_t)rd_be(d + pos, 2);
    r->suf = (uint32_t)rd_be(d + pos + 2, 2);
    pos += 4;
    if ((uint64_t)pos + r->suf + 9 > end) return SDB_CORRUPT_BLOCK;
    r->suf_pos = pos;
    pos += r->suf;
    r->seq = rd_be(d + pos, 8);
    pos += 8;
    uint8_t f = d[pos++];
    if (!flags_ok(f)) return SDB_INVALID_ROW_FLAGS;
    uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > end) return SDB_CORRUPT_BLOCK;
    r->ets = 0;
    r->cts = 0;
    if (f & SDB_FLAG_HAS_EXPIRE_TS) {
        r->ets = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    if (f & SDB_FLAG_HAS_CREATE_TS) {
        r->cts = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    r->vlen = 0;
    r->val_pos = 0;
    r->flags = f;
    if (f & SDB_FLAG_TOMBSTONE) {
        r->flags = (uint8_t)(f & ~SDB_FLAG_HAS_EXPIRE_TS);
    } else {
        if ((uint64_t)pos + 4 > end) return SDB_CORRUPT_BLOCK;
        r->vlen = (uint32_t)rd_be(d + pos, 4);
        pos += 4;
        if ((uint64_t)pos + r->vlen > end) return SDB_CORRUPT_BLOCK;
        r->val_pos = pos;
    }
    return 0;
}

SDB_DEV void wave_sync_d() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Block parse plan shared by count and emit: where the data lives and how rows are split on lanes.
template <typename P>
struct BlockViewT {
    P d;                   // block bytes (LDS or global), CRC stripped
    uint32_t data_end;     // end of rows
    uint32_t count;        // trailer count (restarts for V2, entries for V1)
    P offs;                // trailer offsets (big-endian u16)
    int status;
};
typedef BlockViewT<const uint8_t *> BlockView;
typedef BlockViewT<const lu8 *> LdsBlockView;

// Stage + CRC-check block k; fills the view.  Called by a whole wave.
// check = false (the emit pass: the count pass verified the CRC) skips the CRC.
SDB_DEV BlockView load_block(const DecodeArgs &a, uint64_t k, uint8_t *stage, const uint32_t (*crc)[256], uint32_t cap = kDecCap,
                             bool check = true) {
    BlockView v{};
    const uint64_t s = a.block_off[k], e = block_end_of(a, k);
    const uint64_t len = e - s;
    if (e < s || len < 4) {  // a non-monotone block_off is a corrupt range, never a huge read
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    const uint8_t *g = a.blocks + s;
    const uint32_t blen = (uint32_t)(len - 4);
    uint32_t c;
    const uint8_t *d;
    if (len + 32 <= cap) {
        // 16-byte granules covering [s, e); stage[pad + i] = g[i]
        uint64_t a0 = s & ~15ull, a1 = (e + 15) & ~15ull;
        uint32_t nchunk = (uint32_t)((a1 - a0) >> 4);
        const uint4 *src = (const uint4 *)(a.blocks + a0);
        for (uint32_t q = lane_id(); q < nchunk; q += 64) ((uint4 *)stage)[q] = src[q];
        wave_sync_d();
        d = stage + (s & 15);
        c = blen >= 4 && check ? wave_crc32_lds(d, blen, crc) : 0;
    } else if (!check) {
        c = 0;
        d = g;
    } else {
        // big block: CRC through 4 KiB LDS windows, parse straight from HBM
        uint64_t nwin = (blen + 4095) >> 12;
        uint64_t first = blen - ((nwin - 1) << 12);
        uint32_t acc = 0;
        for (uint64_t w = 0; w < nwin; w++) {
            uint64_t wbeg = (w == 0) ? 0 : first + ((w - 1) << 12);
            uint32_t wlen = (uint32_t)((w == 0) ? first : 4096);
            // the window's 16-byte granules (one load each, all in flight), window byte 0 at stage[gp]
            const uint64_t ga = (s + wbeg) & ~15ull;
            const uint32_t gp = (uint32_t)((s + wbeg) & 15), ng = (gp + wlen + 15) >> 4;
            const uint4 *src = (const uint4 *)(a.blocks + ga);
            for (uint32_t q = lane_id(); q < ng; q += 64) ((uint4 *)stage)[q] = src[q];
            wave_sync_d();
            // crc32fast's init folded into message bytes [0, 4), which may straddle the first two windows
            if (lane_id() < 4 && wbeg + lane_id() < 4 && lane_id() < wlen) stage[gp + lane_id()] ^= 0xFF;
            wave_sync_d();
            uint32_t raw = wave_crc_raw_lds(stage + gp, wlen, crc, false);
            acc = (w == 0) ? raw : (gf_mul(c_shift.window, acc) ^ raw);
            wave_sync_d();
        }
        c = acc ^ 0xFFFFFFFFu;
        d = g;
    }
    if (blen < 4 && check) {  // the wave CRC folds the init into 4 message bytes; tiny blocks go byte-wise
        uint32_t x = 0xFFFFFFFFu;
        for (uint32_t q = 0; q < blen; q++) x = crc[0][(x ^ d[q]) & 0xFF] ^ (x >> 8);
        c = x ^ 0xFFFFFFFFu;
    }
    uint32_t stored = (uint32_t)rd_be(d + blen, 4);
    if (check && c != stored) {
        v.status = SDB_CHECKSUM_MISMATCH;  // validate_checksum (format/sst.rs:1029-1038)
        return v;
    }
    if (blen < 2) {
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    uint32_t cnt = (uint32_t)rd_be(d + blen - 2, 2);  // Block::decode (format/block.rs:28-46)
    if (2 + 2 * (uint64_t)cnt > blen) {
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    v.d = d;
    v.count = cnt;
    v.data_end = blen - 2 - 2 * cnt;
    v.offs = d + v.data_end;
    v.status = 0;
    return v;
}

// Fast path: a block whose CRC input fits one 4 KiB wave image.  The block's 16-byte granules are
// staged so that image byte p0 = s & 15 is block byte 0; the bytes before it and past the CRC input
// (to the end of the last 64-byte segment) are zeroed, crc32fast's init is folded into the first four
// message bytes in place, and the shared wave CRC (sdb_crc.h) runs once; the four bytes are restored
// for the parse.  check = false (the emit pass) only stages.
SDB_DEV bool dec_fast(uint64_t s, uint64_t e) {
    const uint64_t len = e - s;
    return e >= s && len >= 8 && (s & 15) + len <= kDecImg && (s & 15) + len - 4 <= 4096;
}

// A block's 16-byte granules in registers (lane l holds granules l, l + 64, ...): loaded one block
// ahead so the HBM latency overlaps the previous block's work.
constexpr int kGranRegs = 5;  // ceil(kDecImg / 16 / 64)
struct Granules {
    uint4 g[kGranRegs];
};
SDB_DEV void gran_load(const DecodeArgs &a, uint64_t s, uint64_t e, Granules &r) {
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t a0 = s & ~15ull;
    const uint32_t ng = (uint32_t)((((e + 15) & ~15ull) - a0) >> 4);
    const uint4 *src = (const uint4 *)(a.blocks + a0);
#pragma unroll
    for (int i = 0; i < kGranRegs; i++) {
        const uint32_t q = l + 64 * i;
        if (q < ng) r.g[i] = src[q];
    }
}
// The same granules by unconditional loads (lanes past the block re-read its last granule; a block that
// is not dec_fast reads only its first granule): no load sits under a branch, so the compiler's vmcnt
// bookkeeping stays exact and a prefetch is never waited on before its use (see k_emit).
SDB_DEV void gran_load_u(const DecodeArgs &a, uint64_t s, uint64_t e, Granules &r) {
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t a0 = s & ~15ull;
    const uint32_t ng = dec_fast(s, e) ? (uint32_t)((((e + 15) & ~15ull) - a0) >> 4) : 1u;
    const uint4 *src = (const uint4 *)(a.blocks + a0);
#pragma unroll
    for (int i = 0; i < kGranRegs; i++) {
        const uint32_t q = l + 64 * i;
        r.g[i] = src[q < ng ? q : ng - 1];
    }
}
SDB_DEV void gran_store(uint64_t s, uint64_t e, const Granules &r, lu8 *img) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t ng = (uint32_t)((((e + 15) & ~15ull) - (s & ~15ull)) >> 4);
#pragma unroll
    for (int i = 0; i < kGranRegs; i++) {
        const uint32_t q = l + 64 * i;
        if (q < ng) {
            u32x4 w;
            w.x = r.g[i].x;
            w.y = r.g[i].y;
            w.z = r.g[i].z;
            w.w = r.g[i].w;
            ((lu128 *)img)[q] = w;
        }
    }
}

// validate_checksum (format/sst.rs:1029-1038) of a block staged by stage_lds (image byte p0 = block byte
// 0, the 64 bytes before img zero): zero the bytes before p0, fold crc32fast's init into the first four,
// one wave CRC, restore.  Every lane gets the verdict.
SDB_DEV bool crc_staged_ok(lu8 *img, uint32_t p0, uint32_t blen) {
    const uint32_t l = (uint32_t)lane_id();
    const lu8 *d = img + p0;
    const uint32_t stored = ((uint32_t)d[blen] << 24) | ((uint32_t)d[blen + 1] << 16) | ((uint32_t)d[blen + 2] << 8) |
                            (uint32_t)d[blen + 3];
    wave_sync_d();
    if (l < p0) img[l] = 0;
    if (l < 4) img[p0 + l] ^= 0xFF;
    wave_sync_d();
#ifdef SDB_DEC_CRC_SLICE
    const uint32_t c = wave_crc_image_ra(img, p0 + blen);
#else
    const uint32_t c = wave_crc_image_mfma<0, kCrcMfmaTreeKiB>(img, p0 + blen);
#endif
    wave_sync_d();
    if (l < 4) img[p0 + l] ^= 0xFF;
    wave_sync_d();
    return c == stored;
}

SDB_DEV LdsBlockView stage_lds(const DecodeArgs &a, uint64_t s, uint64_t e, lu8 *img, bool check,
                               const Granules *pre = nullptr, bool staged = false) {
    LdsBlockView v{};
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t p0 = (uint32_t)(s & 15), len = (uint32_t)(e - s), blen = len - 4, Lc = p0 + blen;
    if (staged) {  // the caller wrote the granules (gran_store)
    } else if (pre) {
        gran_store(s, e, *pre, img);
    } else {
        Granules g;
        gran_load(a, s, e, g);
        gran_store(s, e, g, img);
    }
    wave_sync_d();
    const lu8 *d = img + p0;
    (void)l;
    (void)Lc;
    if (check && !crc_staged_ok(img, p0, blen)) {
        v.status = SDB_CHECKSUM_MISMATCH;  // validate_checksum (format/sst.rs:1029-1038)
        return v;
    }
    const uint32_t cnt = (uint32_t)rd_be(d + blen - 2, 2);  // Block::decode (format/block.rs:28-46)
    if (2 + 2 * (uint64_t)cnt > blen) {
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    v.d = d;
    v.count = cnt;
    v.data_end = blen - 2 - 2 * cnt;
    v.offs = d + v.data_end;
    v.status = 0;
    return v;
}

// LDS -> LDS byte copy, eight bytes in flight per step (one wait per step, not per byte).
SDB_DEV void lds_copy_small(lu8 *dst, const lu8 *src, uint32_t n) {
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint8_t t[8];
#pragma unroll
        for (int q = 0; q < 8; q++) t[q] = src[i + q];
#pragma unroll
        for (int q = 0; q < 8; q++) dst[i + q] = t[q];
    }
    for (; i < n; i++) dst[i] = src[i];
}

// Store LDS bytes kbuf[o .. o + n) to global [g, g + n), o = g & 15: 16-byte stores for the granules
// inside the range, byte stores at its two edges (neighbouring blocks' keys share those granules).
SDB_DEV void wave_store_bytes(uint8_t *g, const lu8 *kbuf, uint64_t n) {
    if (!n) return;
    const uintptr_t d0 = (uintptr_t)g, d1 = d0 + n;
    const uintptr_t a0 = d0 & ~(uintptr_t)15, a1 = (d1 + 15) & ~(uintptr_t)15;
    const uint32_t nch = (uint32_t)((a1 - a0) >> 4);
    for (uint32_t c = lane_id(); c < nch; c += 64) {
        const uintptr_t ga = a0 + 16 * (uintptr_t)c;
        const lu8 *li = kbuf + 16 * c;
        if (ga >= d0 && ga + 16 <= d1) {
            const u32x4 w = *(const lu128 *)li;
            // global, not flat: a flat store counts in both wait counters and forces the compiler's waits to 0
            *(__attribute__((address_space(1))) u32x4 *)ga = w;
        } else {
            // an edge granule (shared with the neighbouring block's keys): bytes [s, e) of it as at most
            // four unaligned 8 / 4 / 2 / 1-byte stores instead of a store per byte
            const u32x4 w = *(const lu128 *)li;
            const uint32_t s = ga >= d0 ? 0u : (uint32_t)(d0 - ga), e = ga + 16 <= d1 ? 16u : (uint32_t)(d1 - ga);
            uint64_t lo = (uint64_t)w.x | ((uint64_t)w.y << 32), hi = (uint64_t)w.z | ((uint64_t)w.w << 32);
            if (s >= 8) {
                lo = hi >> (8 * (s - 8));
                hi = 0;
            } else if (s) {
                lo = (lo >> (8 * s)) | (hi << (64 - 8 * s));
                hi >>= 8 * s;
            }
            typedef __attribute__((address_space(1))) uint8_t gu8;
            gu8 *dst = (gu8 *)ga + s;
            const uint32_t n = e - s, b8 = n & 8, b4 = n & 4, b2 = n & 2;
            typedef __attribute__((address_space(1))) uint64_t u64u __attribute__((aligned(1)));
            typedef __attribute__((address_space(1))) uint32_t u32u __attribute__((aligned(1)));
            typedef __attribute__((address_space(1))) uint16_t u16u __attribute__((aligned(1)));
            if (b8) *(u64u *)dst = lo;
            const uint64_t t = b8 ? hi : lo;
            if (b4) *(u32u *)(dst + b8) = (uint32_t)t;
            if (b2) *(u16u *)(dst + b8 + b4) = (uint16_t)(t >> (8 * b4));
            if (n & 1) dst[b8 + b4 + b2] = (uint8_t)(t >> (8 * (b4 + b2)));
        }
    }
}

// V2 plan: lane q parses restart region q when the block is "regular" (restart 0 at offset 0,
// strictly increasing restarts, regions ending exactly on the next restart, shared == 0 at every
// region start); otherwise lane 0 walks the whole block like BlockIteratorV2::next does.
// Returns (entries, key bytes, status) reduced over the wave.
struct Tally {
    uint64_t entries, key_bytes;
    int status;
    bool sequential;
};

template <typename P>
SDB_DEV Tally tally_v2(const BlockViewT<P> &v) {
    Tally t{0, 0, 0, false};
    const int l = lane_id();
    const uint32_t R = v.count;
    bool regular = R > 0 && rd_be(v.offs, 2) == 0;
    uint32_t my_entries = 0, my_kb = 0;
    int my_status = 0;
    bool my_regular = true;
    for (uint32_t q = l; q < R && regular; q += 64) {
        uint32_t pos = (uint32_t)rd_be(v.offs + 2 * q, 2);
        uint32_t end = (q + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * q + 2, 2) : v.data_end;
        if (end <= pos || end > v.data_end) {
            my_regular = false;
            break;
        }
        uint32_t prevlen = 0;
        bool firstrow = true;
        while (pos < end) {
            RowV2 r;
            int st = parse_v2(v.d, v.data_end, pos, &r);
            if (st) {
                my_status = st;
                break;
            }
            if (firstrow && r.shared != 0) my_regular = false;
            if (!firstrow && r.shared > prevlen) {
                my_status = SDB_CORRUPT_BLOCK;
                break;
            }
            firstrow = false;
            prevlen = r.shared + r.unshared;
            my_entries++;
            my_kb += prevlen;
            pos = r.next;
        }
        if (pos != end && !my_status) my_regular = false;
        if (my_status || !my_regular) break;
    }
    // wave-reduce: regular only if every lane stayed regular
    bool all_regular = regular && (__ballot(!my_regular) == 0);
    if (all_regular) {
        // lowest-lane error wins (rows are in lane order within the block)
        uint64_t bad = __ballot(my_status != 0);
        if (bad) {
            int first = __builtin_ctzll(bad);
            t.status = __shfl(my_status, first, 64);
            return t;
        }
        t.entries = wave_sum((uint64_t)my_entries);
        t.key_bytes = wave_sum((uint64_t)my_kb);
        return t;
    }
    // sequential walk (lane 0)
    t.sequential = true;
    uint64_t ent = 0, kb = 0;
    int st = 0;
    if (l == 0) {
        uint32_t curlen = 0;
        if (R > 0) {  // decode_first_key_at_restart(0) asserts shared == 0
            uint32_t p = (uint32_t)rd_be(v.offs, 2);
            uint32_t sh = 0, un = 0, vl = 0;
            if (!rd_varint(v.d, v.data_end, &p, &sh) || !rd_varint(v.d, v.data_end, &p, &un) ||
                !rd_varint(v.d, v.data_end, &p, &vl) || sh != 0 || (uint64_t)p + un > v.data_end)
                st = SDB_CORRUPT_BLOCK;
            curlen = un;
        }
        uint32_t pos = 0;
        while (!st && pos < v.data_end) {
            RowV2 r;
            st = parse_v2(v.d, v.data_end, pos, &r);
            if (st) break;
            if (r.shared > curlen) {
                st = SDB_CORRUPT_BLOCK;
                break;
            }
            curlen = r.shared + r.unshared;
            ent++;
            kb += curlen;
            pos = r.next;
        }
    }
    t.status = __shfl(st, 0, 64);
    t.entries = __shfl(ent, 0, 64);
    t.key_bytes = __shfl(kb, 0, 64);
    return t;
}

// Regular V2 blocks staged in LDS, fast path: each region lane walks its rows reading only the header
// (one 4-byte window: single-byte varints) and stepping by hdr + unshared + vlen + 9, i.e. assuming no
// timestamps; every row's flags byte is read off the critical path and checked after the walk.  Any
// multi-byte varint, timestamp or bad flag sends the block to the exact walk (tally_v2).
SDB_DEV uint32_t lds_read4(const lu8 *p) {
    const uint32_t addr = lds_addr((const void *)p), sh = addr & 3;
    const lu32 *d = (const lu32 *)(uintptr_t)(addr & ~3u);
    return __builtin_amdgcn_alignbyte(d[1], d[0], sh);
}

SDB_DEV uint32_t lds_byte(const lu8 *p) { return *p; }

// The region walks as one wave-uniform loop (no per-lane breaks: a lane that finishes or fails just
// stops advancing), so a step is ~20 instructions instead of ~80 of exec-mask bookkeeping and branches
// (the walk was issue-bound with 1 - 4 live lanes per wave).
SDB_DEV bool tally_v2_fast(const LdsBlockView &v, Tally &t, uint16_t *rowpos, uint64_t *rcnt) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t R = v.count;
    if (R == 0 || R > 64 || rd_be(v.offs, 2) != 0) return false;
    uint32_t p = 0, end = 0, bad = 0;
    if (l < R) {
        p = (uint32_t)rd_be(v.offs + 2 * l, 2);
        end = (l + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * l + 2, 2) : v.data_end;
        if (end <= p || end > v.data_end) bad = 1;
    }
    uint32_t ne = 0, kb = 0, kmax = 0, prevlen = 0, fl = 0;
    const uint32_t rec = (rowpos && l < 4) ? 32u : 0u;  // positions recorded for regions 0..3, <= 32 rows each
    uint16_t *rp = rowpos + 32 * l;
    // every condition below is bit arithmetic on 0/1 values (no short-circuit), so the step compiles
    // to straight-line selects; the only branches are the loop's and the position store's
    constexpr uint32_t kFlagsOk = (1u << 0) | (1u << SDB_FLAG_TOMBSTONE) | (1u << SDB_FLAG_MERGE_OPERAND);
    for (;;) {
        const uint32_t act = (uint32_t)(p < end) & (bad ^ 1u);
        if (__ballot(act != 0) == 0) break;
        const uint32_t h = lds_read4(v.d + p);
        const uint32_t sh = h & 0xFF, un = (h >> 8) & 0xFF, vl = (h >> 16) & 0xFF;
        const uint32_t nx = p + 12 + un + vl, klen = sh + un;
        // the previous row's flags (read one step earlier): value, tombstone or merge only
        const uint32_t fbad = (((kFlagsOk >> (fl & 31)) & 1u) ^ 1u) | (uint32_t)(fl > 31);
        const uint32_t lim = ne ? prevlen : 0u;
        const uint32_t rbad = (uint32_t)((h & 0x808080u) != 0) | (uint32_t)(sh > lim) | (uint32_t)(nx > end);
        const uint32_t fpos = nx - 1 < end ? nx - 1 : end;
        const uint32_t fnew = lds_byte(v.d + fpos);
        if (act && ne < rec) rp[ne] = (uint16_t)p;
        bad = act ? (fbad | rbad) : bad;
        fl = act ? fnew : fl;
        kmax = act && klen > kmax ? klen : kmax;
        kb += act ? klen : 0u;
        prevlen = act ? klen : prevlen;
        ne += act;
        p = act ? nx : p;
    }
    bad |= (fl != 0 && fl != SDB_FLAG_TOMBSTONE && fl != SDB_FLAG_MERGE_OPERAND) ? 1u : 0u;
    if (p != end) bad = 1;
    if (__ballot(l < R && bad) != 0) return false;
    t.entries = wave_sum((uint64_t)ne);
    t.key_bytes = wave_sum((uint64_t)kb);
    t.status = 0;
    t.sequential = false;
    // the emit pass parses lane = row straight from the recorded positions when the block has <= 4
    // regions of <= 32 rows, <= 64 rows and keys of <= 16 bytes
    const uint32_t mx = wave_max(l < R ? ne : 0u), kmx = wave_max(kmax);
    uint64_t c = ~0ull;
    if (R <= 4 && mx <= 32 && t.entries <= 64 && kmx <= 16) {
        c = 0;
        for (uint32_t q = 0; q < R; q++) c |= (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)ne, (int)q) << (16 * q);
    }
    if (l == 0 && rcnt) *rcnt = c;
    return true;
}

// Speculative lane-per-row parse of a block of <= 4 restart regions (the common 4 KiB shape: 16-row
// restart intervals give 3 regions).  Lane group q (G = 64 / 16 / ... lanes) takes region q, lane i of
// it row i.  Row positions are guessed from the lengths of rows 0 and 1 (c_i = p_1 + (i - 1) L_1), every
// lane reads its header, and the guesses are checked against the previous lane's row end; the first
// wrong guess of a group shifts the guesses after it by its error (right for a single row of another
// length, e.g. a key-counter carry), for at most four rounds.  The fixed point is exactly the walk of
// BlockIteratorV2::next (block_iterator_v2.rs:235-267) over regular rows; anything else (no
// convergence, more rows than lanes, multi-byte varints, timestamps, bad flags) returns false and the
// caller walks the block.  All lanes work, vs 1 - 4 lanes stepping row by row.
SDB_DEV uint32_t bperm(uint32_t lane, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lane << 2), (int)v); }

SDB_DEV bool tally_v2_spec(const LdsBlockView &v, Tally &t, uint16_t *rowpos, uint64_t *rcnt) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t R = v.count;
    if (R == 0 || R > 4 || rd_be(v.offs, 2) != 0) return false;
    const uint32_t lg = R == 1 ? 6u : (R == 2 ? 5u : 4u), G = 1u << lg;
    const uint32_t q = l >> lg, i = l & (G - 1);
    const bool grp = q < R;
    const uint64_t gmask = lg == 6 ? ~0ull : (((1ull << G) - 1) << (q * G));
    uint32_t pos = 0, end = 0;
    if (grp) {
        pos = (uint32_t)rd_be(v.offs + 2 * q, 2);
        end = (q + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * q + 2, 2) : v.data_end;
    }
    if (__ballot(grp && (end <= pos || end > v.data_end)) != 0) return false;
    constexpr uint32_t kEnd = 0xFFFFFFFFu;
    // initial guesses from the lengths of rows 0 and 1 (reads shared by the group's lanes)
    const uint32_t h0 = lds_read4(v.d + (grp ? pos : 0u));
    const uint32_t p1 = pos + 12 + ((h0 >> 8) & 0xFF) + ((h0 >> 16) & 0xFF);
    const uint32_t h1 = lds_read4(v.d + (grp && p1 < end ? p1 : 0u));
    const uint32_t L1 = 12 + ((h1 >> 8) & 0xFF) + ((h1 >> 16) & 0xFF);
    uint32_t c = i == 0 ? pos : p1 + (i - 1) * L1;
    uint32_t h = 0, n = 0, live = 0;
    for (int round = 0;; round++) {
        live = grp && c < end ? 1u : 0u;
        h = lds_read4(v.d + (live ? c : 0u));
        n = c + 12 + ((h >> 8) & 0xFF) + ((h >> 16) & 0xFF);
        const uint32_t n_prev = bperm(l - 1, n), live_prev = bperm(l - 1, live);
        const uint32_t exp = i == 0 ? pos : (live_prev && n_prev < end ? n_prev : kEnd);
        const bool mism = grp && (exp == kEnd ? live != 0 : c != exp);
        const uint64_t M = __ballot(mism);
        if (M == 0) break;
        if (round == 3) return false;
        const uint64_t mg = M & gmask;
        const uint32_t f = mg ? (uint32_t)__builtin_ctzll(mg) : 0u;
        const uint32_t fe = bperm(f, exp), fc = bperm(f, c);
        if (mg && l >= f) c = fe == kEnd ? kEnd : c + (fe - fc);
    }
    // the converged rows: fast shape and regular
    const uint32_t sh = h & 0xFF, un = (h >> 8) & 0xFF, klen = sh + un;
    const uint32_t kprev = bperm(l - 1, klen);
    const uint32_t fl = lds_byte(v.d + (live ? n - 1 : 0u));
    constexpr uint32_t kFlagsOk = (1u << 0) | (1u << SDB_FLAG_TOMBSTONE) | (1u << SDB_FLAG_MERGE_OPERAND);
    const bool rbad = (h & 0x808080u) != 0 || n > end || (i == 0 ? sh != 0 : sh > kprev) || fl > 31 ||
                      !((kFlagsOk >> (fl & 31)) & 1u) || (i == G - 1 && n < end);
    if (__ballot(live && rbad) != 0) return false;
    const uint64_t L = __ballot(live != 0);
    t.entries = (uint64_t)__builtin_popcountll(L);
    t.key_bytes = wave_sum((uint64_t)(live ? klen : 0u));
    t.status = 0;
    t.sequential = false;
    if (rowpos && live && q < 4 && i < 32) rowpos[32 * q + i] = (uint16_t)c;
    // per-region row counts for the emit pass's lane-per-row parse (<= 64 rows, keys of <= 16 bytes)
    const uint32_t kmx = wave_max(live ? klen : 0u);
    uint64_t rc = ~0ull;
    if (kmx <= 16) {
        rc = 0;
        for (uint32_t r = 0; r < R; r++) {
            const uint64_t gm = lg == 6 ? ~0ull : (((1ull << G) - 1) << (r * G));
            const uint32_t cnt = (uint32_t)__builtin_popcountll(L & gm);
            rc |= (uint64_t)cnt << (16 * r);
            if (cnt > 32) rc = ~0ull;  // positions are recorded for 32 rows per region
            if (cnt > 32) break;
        }
    }
    if (l == 0 && rcnt) *rcnt = rc;
    return true;
}

template <typename P>
SDB_DEV Tally tally_v1(const BlockViewT<P> &v) {
    Tally t{0, 0, 0, false};
    const int l = lane_id();
    const uint32_t R = v.count;
    if (R == 0) return t;
    // decode_first_key (block_iterator.rs:235-242)
    if (v.data_end < 4 || rd_be(v.d, 2) != 0 || 4 + rd_be(v.d + 2, 2) > v.data_end) {
        t.status = SDB_CORRUPT_BLOCK;
        return t;
    }
    const uint32_t fk = (uint32_t)rd_be(v.d + 2, 2);
    uint64_t kb = 0;
    int st = 0;
    uint64_t bad_first = ~0ull;
    for (uint32_t i = l; i < R; i += 64) {
        RowV0 r;
        int s = parse_v0(v.d, v.data_end, (uint32_t)rd_be(v.offs + 2 * i, 2), &r);
        if (!s && r.prefix > fk) s = SDB_CORRUPT_BLOCK;
        if (s) {
            if (i < bad_first) {
                bad_first = i;
                st = s;
            }
            continue;
        }
        kb += r.prefix + r.suf;
    }
    // lowest failing entry wins
    uint64_t mn = bad_first;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint64_t o = __shfl_xor(mn, d, 64);
        mn = o < mn ? o : mn;
    }
    if (mn != ~0ull) {
        uint64_t owner = __ballot(bad_first == mn);
        t.status = __shfl(st, __builtin_ctzll(owner), 64);
        return t;
    }
    t.entries = R;
    t.key_bytes = wave_sum(kb);
    return t;
}

// Descending iteration (DescendingBlockIteratorV2, block_iterator_v2.rs:318-430) decodes each restart
// region from its restart (asserting shared == 0 there, :71-93) and yields it in reverse.  For a
// regular block (regions that start at restarts with shared == 0 and end exactly at the next one)
// that is the ascending decode reversed; a block without restarts yields nothing; any other layout
// is reported as SDB_CORRUPT_BLOCK (the reference would assert or read rows across regions).
SDB_DEV void desc_rule(uint32_t restarts, Tally &t) {
    if (t.status) return;
    if (restarts == 0) {
        t.entries = t.key_bytes = 0;
        t.sequential = false;
    } else if (t.sequential) {
        t.status = SDB_CORRUPT_BLOCK;
    }
}

// --- blocks over one wave image (SstBlockSize 8 - 64 KiB): restart-region pieces --------------------
// A regular V2 block is cut into pieces of consecutive restart regions (<= 64 regions, <= kPieceBytes
// bytes): each piece is staged in the wave's LDS image (16-byte granules) with its region offsets
// rebased into a small big-endian table after the data, and parsed there by the same LDS walks as a
// small block.  Region boundaries reset the key prefix (shared == 0), so pieces are independent.  Not
// applicable (nothing staged, false): the first region does not start at 0, or a region is longer than
// a piece; the caller then walks the block from HBM as before.
constexpr uint32_t kPieceBytes = 3968, kPieceOffs = 4000;  // piece data in img[0, 3999], offsets at 4000
static_assert(kPieceOffs + 128 <= kDecImg && 15 + kPieceBytes + 16 <= kPieceOffs, "piece layout");
SDB_DEV uint32_t region_off(const BlockView &v, uint32_t q) { return (uint32_t)rd_be(v.offs + 2 * q, 2); }
template <typename F>
SDB_DEV bool for_each_piece(const DecodeArgs &a, uint64_t s, const BlockView &v, lu8 *img, F f) {
    const uint32_t l = (uint32_t)lane_id(), R = v.count;
    // only blocks parsed from HBM: a block load_block staged whole lives in this same LDS image (its
    // trailer offsets would be overwritten by the first piece) and is walked there instead
    if (v.d != a.blocks + s) return false;
    if (R == 0 || region_off(v, 0) != 0) return false;
    for (uint32_t q0 = 0; q0 < R; q0 += 64) {
        const uint32_t q = q0 + l;
        const uint32_t lo = q < R ? region_off(v, q) : 0, hi = q < R ? (q + 1 < R ? region_off(v, q + 1) : v.data_end) : 0;
        if (__ballot(q < R && (hi < lo || hi - lo > kPieceBytes)) != 0) return false;
    }
    for (uint32_t qa = 0; qa < R;) {
        const uint32_t q = qa + l;
        const uint32_t base = region_off(v, qa);
        const uint32_t lo = q < R ? region_off(v, q) : 0, hi = q < R ? (q + 1 < R ? region_off(v, q + 1) : v.data_end) : 0;
        const uint64_t fit = __ballot(q < R && hi >= base && hi - base <= kPieceBytes);
        const uint32_t m = fit == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~fit);  // regions qa .. qa + m - 1
        const uint32_t pb = (uint32_t)__builtin_amdgcn_readlane((int)hi, (int)(m - 1));
        const uint64_t g0 = s + base, ga = g0 & ~15ull;
        const uint32_t p0 = (uint32_t)(g0 & 15), ng = (p0 + (pb - base) + 15) >> 4;
        const uint4 *src = (const uint4 *)(a.blocks + ga);
        for (uint32_t x = l; x < ng; x += 64) {
            const uint4 w4 = src[x];
            u32x4 w;
            w.x = w4.x;
            w.y = w4.y;
            w.z = w4.z;
            w.w = w4.w;
            ((lu128 *)img)[x] = w;
        }
        if (l < m) {
            const uint32_t r = lo - base;
            img[kPieceOffs + 2 * l] = (uint8_t)(r >> 8);
            img[kPieceOffs + 2 * l + 1] = (uint8_t)r;
        }
        wave_sync_d();
        LdsBlockView pv{};
        pv.d = img + p0;
        pv.data_end = pb - base;
        pv.count = m;
        pv.offs = img + kPieceOffs;
        pv.status = 0;
        if (!f(pv, base)) return true;  // the callback stops the walk
        wave_sync_d();
        qa += m;
    }
    return true;
}

// Count pass of a big V2 block by pieces: false when not applicable or when a piece is irregular (the
// whole-block walk then decides, exactly as before).
SDB_DEV bool tally_v2_pieces(const DecodeArgs &a, uint64_t s, const BlockView &v, lu8 *img, Tally &t) {
    Tally acc{0, 0, 0, false};
    bool irregular = false;
    const bool ok = for_each_piece(a, s, v, img, [&](const LdsBlockView &pv, uint32_t) {
        // the small-block walks first (regular rows; no positions recorded), the general one decides the rest
        Tally pt{0, 0, 0, false};
        if (!tally_v2_spec(pv, pt, nullptr, nullptr) && !tally_v2_fast(pv, pt, nullptr, nullptr)) pt = tally_v2(pv);
        // an irregular piece, or a row that fails to parse against the piece's end (it may run on into the
        // next piece, which the whole-block walk reads as an irregular block): the whole-block walk decides
        if (pt.sequential || pt.status) {
            irregular = true;
            return false;
        }
        acc.entries += pt.entries;
        acc.key_bytes += pt.key_bytes;
        return true;
    });
    if (!ok || irregular) return false;
    t = acc;
    return true;
}

// Per-block flag bits (DecodeArgs::flag), written by the count passes, read by the emit passes.
constexpr uint8_t kFlagSeq = 1;  // V2 block walked sequentially (irregular restart regions)
constexpr uint8_t kFlagGen = 2;  // emitted by k_dec_emit_gen (V1, rows not recorded, keys over the row table, big)
constexpr uint8_t kFlagBig = 4;  // over one wave image: counted by k_dec_count_big
constexpr uint8_t kFlagBad = 8;  // failed in a count pass (its checksum already verified there)

// The blocks of wave w in the passes that pick flagged blocks ([k0, k1), contiguous): the flags are
// read 64 at a time (one byte per lane) and the flagged blocks taken in order from the ballot.
template <typename F>
SDB_DEV void for_flagged(const DecodeArgs &a, uint8_t bit, uint64_t gwave, uint64_t nwaves, F f) {
    const uint64_t per = (a.nblocks + nwaves - 1) / nwaves, k0 = gwave * per;
    const uint64_t k1 = k0 + per < a.nblocks ? k0 + per : a.nblocks;
    for (uint64_t b = k0; b < k1; b += 64) {
        const uint64_t k = b + lane_id();
        uint64_t m = __ballot(k < k1 && (a.flag[k] & bit));
        while (m) {
            const uint32_t i = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            f(b + i);
        }
    }
}

// Whether any block of this workgroup's waves' ranges (for_flagged) carries `bit`: a workgroup without
// one returns before it stages anything (the common case: a run of 4 KiB blocks has none).  scratch:
// 16 dwords of the caller's dynamic LDS, free until the caller stages (__syncthreads_or would add
// static LDS and move the dynamic region off address 0, where the CRC lookups expect their tables).
SDB_DEV bool wg_any_flagged(const DecodeArgs &a, uint8_t bit, uint32_t *scratch) {
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6), per = (a.nblocks + nwaves - 1) / nwaves;
    const uint64_t k0 = (uint64_t)blockIdx.x * (blockDim.x >> 6) * per;
    const uint64_t k1 = k0 + (blockDim.x >> 6) * per < a.nblocks ? k0 + (blockDim.x >> 6) * per : a.nblocks;
    bool any = false;
    for (uint64_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) any |= (a.flag[k] & bit) != 0;
    const bool wany = __ballot(any) != 0;
    if (lane_id() == 0) scratch[threadIdx.x >> 6] = wany ? 1u : 0u;
    __syncthreads();
    uint32_t r = 0;
    for (uint32_t q = 0; q < (blockDim.x >> 6); q++) r |= scratch[q];
    __syncthreads();
    return r != 0;
}

SDB_DEV void count_result(const DecodeArgs &a, uint64_t k, const Tally &t, uint8_t gen) {
    if (lane_id() != 0) return;
    if (t.status) {
        a.cnt[k] = 0;
        a.kbytes[k] = 0;
        a.flag[k] = kFlagBad;
        atomicMin(a.err, (unsigned long long)((k << 8) | (uint64_t)t.status));
        unsigned long long slot = atomicAdd(a.nbad, 1ull);
        if (slot < a.bad_cap) a.bad_block[slot] = (uint32_t)k;
    } else {
        a.cnt[k] = t.entries;
        a.kbytes[k] = t.key_bytes;
        a.flag[k] = (uint8_t)((t.sequential ? kFlagSeq : 0) | gen);
    }
}

// D1 count, blocks of one wave image (dec_fast); the others are flagged kFlagBig for k_dec_count_big.
// A block the lane-per-row emit takes (V2, rows recorded, keys within the row table) is left unflagged;
// the rest are flagged kFlagGen.  LDS: the CRC tables at address 0 (sdb_crc.h: this kernel has no
// static LDS), then one region of kCntWaveLds per wave.
__global__ __launch_bounds__(kCntThreads) __attribute__((amdgpu_waves_per_eu(kCntEu))) void k_dec_count(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (lds_addr((const void *)smem) != 0) {  // sdb_crc.h's lookups assume the tables at LDS address 0
        if (threadIdx.x == 0) atomicMin(a.err, (unsigned long long)SDB_DEVICE_ERROR);
        return;
    }
    dec_crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    lu8 *img = (lu8 *)smem + kDecTabLds + wave * kCntWaveLds + kDecGuard;
    if (lane_id() < kDecGuard / 4) ((lu32 *)(img - kDecGuard))[lane_id()] = 0;  // never written again
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    (void)gwave;
    // software pipeline: block k's granules landed, block k + nwaves's in flight (its offsets landed one
    // block earlier), the offsets of block k + 2 nwaves in flight; unconditional loads and result stores,
    // so the compiler's only vmcnt waits are the hand-overs at the end of an iteration
    uint64_t k = gwave;
    if (k >= a.nblocks) return;
    const uint64_t last = a.nblocks - 1;
    auto clampk = [&](uint64_t x) { return x < a.nblocks ? x : last; };
    uint64_t s = a.block_off[k], e = block_end_of(a, k);
    uint64_t s1 = a.block_off[clampk(k + nwaves)], e1 = block_end_of(a, clampk(k + nwaves));
    Granules cur;
    gran_load_u(a, s, e, cur);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the pipeline starts with nothing in flight
    for (;;) {
        Granules nxt;
        gran_load_u(a, s1, e1, nxt);
        const uint64_t k2 = clampk(k + 2 * nwaves);
        const uint64_t s2 = a.block_off[k2], e2 = block_end_of(a, k2);
        DEC_T(t0);
        Tally t{0, 0, 0, false};
        const bool fast = dec_fast(s, e);
        uint64_t rcv = ~0ull;  // per-region row counts when the rows are recorded (tally_v2_spec / _fast)
        if (fast) {
            // fail-fast: the emit pass verifies the checksums (a block that fails here is checked now, so a
            // corrupt block reports CHECKSUM_MISMATCH before anything its rows would raise)
            const LdsBlockView v = stage_lds(a, s, e, img, !a.fail_fast, &cur);
            DEC_T(t1);
            t.status = v.status;
            if (!v.status) {
                if (a.version == 1) t = tally_v1(v);
                else if (!tally_v2_spec(v, t, a.rowpos + 128 * k, &rcv) && !tally_v2_fast(v, t, a.rowpos + 128 * k, &rcv))
                    t = tally_v2(v);
                if (a.descending && a.version == 2) desc_rule(v.count, t);
            }
            if (a.fail_fast && t.status && !crc_staged_ok(img, (uint32_t)(s & 15), (uint32_t)(e - s - 4)))
                t.status = SDB_CHECKSUM_MISMATCH;
            DEC_T(t2);
            DEC_ACC(0, 0, t1 - t0);
            DEC_ACC(0, 1, t2 - t1);
            DEC_ACC(0, 3, 1);
            wave_sync_d();
        }
        // the block's results: every lane stores lane 0's values (one write per address), unconditionally
        const int st = __builtin_amdgcn_readfirstlane(t.status);
        const uint64_t ent = wave_readlane(t.entries, 0), kb = wave_readlane(t.key_bytes, 0);
        const bool seq = __builtin_amdgcn_readfirstlane((int)t.sequential) != 0;
        rcv = wave_readlane(rcv, 0);  // (the tally functions set it in lane 0)
        uint8_t gen = kFlagGen;
        if (fast && a.version == 2 && !seq && kb + 16 <= kRowTmp && rcv != ~0ull) gen = 0;
        a.rcnt[k] = rcv;
        a.cnt[k] = st || !fast ? 0 : ent;
        a.kbytes[k] = st || !fast ? 0 : kb;
        a.flag[k] = !fast ? kFlagBig : st ? kFlagBad : (uint8_t)((seq ? kFlagSeq : 0) | gen);
        if (st && fast && lane_id() == 0) {
            atomicMin(a.err, (unsigned long long)((k << 8) | (uint64_t)st));
            unsigned long long slot = atomicAdd(a.nbad, 1ull);
            if (slot < a.bad_cap) a.bad_block[slot] = (uint32_t)k;
        }
        wave_sync_d();
        k += nwaves;
        if (k >= a.nblocks) break;
        cur = nxt;
        s = s1;
        e = e1;
        s1 = s2;
        e1 = e2;
    }
}

// D1 count of the blocks over one wave image (kFlagBig): CRC through LDS windows, rows parsed from HBM
// or as restart-region pieces staged in LDS.  Every such block is emitted by k_dec_emit_gen.
__global__ __launch_bounds__(kCntThreads) __attribute__((amdgpu_waves_per_eu(kCntEu))) void k_dec_count_big(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (!wg_any_flagged(a, kFlagBig, (uint32_t *)smem)) return;
    if (lds_addr((const void *)smem) != 0) {
        if (threadIdx.x == 0) atomicMin(a.err, (unsigned long long)SDB_DEVICE_ERROR);
        return;
    }
    crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t(*crc)[256] = (const uint32_t(*)[256])smem;
    const uint32_t wave = threadIdx.x >> 6;
    lu8 *img = (lu8 *)smem + kCrcTablesLds + wave * kCntWaveLds + kDecGuard;
    if (lane_id() < kDecGuard / 4) ((lu32 *)(img - kDecGuard))[lane_id()] = 0;
    uint8_t *stage = (uint8_t *)img;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    for_flagged(a, kFlagBig, gwave, nwaves, [&](uint64_t k) {
        const uint64_t s = a.block_off[k];
        Tally t{0, 0, 0, false};
        const BlockView v = load_block(a, k, stage, crc, kDecImg);
        t.status = v.status;
        if (!v.status) {
            if (a.version == 1) t = tally_v1(v);
            else if (!tally_v2_pieces(a, s, v, img, t)) t = tally_v2(v);
        }
        if (!v.status && a.descending && a.version == 2) desc_rule(v.count, t);
        count_result(a, k, t, kFlagGen);
        wave_sync_d();
    });
}

// --- emit -----------------------------------------------------------------------------------------
// Columns of one entry.  Timestamps are written only when the row carries them (the contract:
// create_ts / expire_ts are valid iff the flag is set).  Descending order (DescendingBlockIteratorV2 /
// BlockIterator Descending yield a block's entries last to first, sst_iter.rs:557 the blocks last to
// first): entry idx of the ascending order is entry N - 1 - idx, and the key at ascending arena position
// kpos lands at KB - kpos - klen, so the arena holds the keys in descending order, each one forward.
SDB_DEV void put_entry(const DecodeArgs &a, uint64_t idx, uint64_t kpos, uint32_t klen, uint64_t vref, uint32_t vlen,
                       uint64_t seq, uint8_t flags, int64_t cts, int64_t ets) {
    if (a.descending) {
        idx = a.dn - 1 - idx;
        kpos = a.dkb - kpos - klen;
    }
    a.out.key_off[idx] = kpos;
    a.out.val_off[idx] = vlen ? vref : 0;
    a.out.val_len[idx] = vlen;
    a.out.seq[idx] = seq;
    a.out.flags[idx] = flags;
    if (flags & SDB_FLAG_HAS_CREATE_TS) a.out.create_ts[idx] = cts;
    if (flags & SDB_FLAG_HAS_EXPIRE_TS) a.out.expire_ts[idx] = ets;
}

// The arena address of the key at ascending position kp (kl bytes): mirrored in descending order.
SDB_DEV uint8_t *key_dst(const DecodeArgs &a, uint64_t kp, uint32_t kl) {
    return a.out.key_arena + (a.descending ? a.dkb - kp - kl : kp);
}
// Descending order: a key its lane just restored in LDS, stored by that lane to its mirrored place (the
// block's keys are not one ascending range there, so no wave_store_bytes).
SDB_DEV void key_store_desc(const DecodeArgs &a, uint64_t kp, const lu8 *src, uint32_t kl) {
    typedef uint32_t u32u __attribute__((aligned(1)));
    uint8_t *g = key_dst(a, kp, kl);
    uint32_t i = 0;
    for (; i + 4 <= kl; i += 4)
        *(u32u *)(g + i) = (uint32_t)src[i] | ((uint32_t)src[i + 1] << 8) | ((uint32_t)src[i + 2] << 16) |
                           ((uint32_t)src[i + 3] << 24);
    for (; i < kl; i++) g[i] = src[i];
}

// Keys of <= 16 bytes as two little-endian u64 (byte x at bits 8x): key = cur[:shared] ++ suffix, the
// suffix a 16-byte window (restore_full_key, row_codec_v2.rs:83-89, on the VALU).  Bytes past the key
// are garbage.
SDB_DEV void key16_merge(uint64_t &lo, uint64_t &hi, uint32_t shared, const uint32_t (&w)[4]) {
    const uint64_t slo = (uint64_t)w[0] | ((uint64_t)w[1] << 32), shi = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    const uint32_t b = 8 * shared;  // 0 .. 128
    uint64_t tlo, thi, mlo, mhi;    // suffix << b; mask of the kept prefix bytes
    if (b == 0) {
        tlo = slo;
        thi = shi;
        mlo = mhi = 0;
    } else if (b < 64) {
        tlo = slo << b;
        thi = (shi << b) | (slo >> (64 - b));
        mlo = ~0ull >> (64 - b);
        mhi = 0;
    } else {
        tlo = 0;
        thi = b < 128 ? slo << (b - 64) : 0;
        mlo = ~0ull;
        mhi = b == 64 ? 0 : (b >= 128 ? ~0ull : ~0ull >> (128 - b));
    }
    lo = (lo & mlo) | (tlo & ~mlo);
    hi = (hi & mhi) | (thi & ~mhi);
}

// V2 emit of one block (BlockIteratorV2 ascending, block_iterator_v2.rs:235-267; restore_full_key,
// row_codec_v2.rs:83-89).  Keys are restored into `kb` (LDS, the block's keys at kb + (kb0 & 15) + rel)
// when kbuf is set, else straight into the arena.  Regular blocks: lane q walks restart region q (a
// wave scan over the regions gives each lane its first entry and key position); otherwise lane 0 walks
// the block.
template <typename P>
SDB_DEV void emit_v2(const DecodeArgs &a, const BlockViewT<P> &v, bool sequential, uint64_t ent0, uint64_t kb0,
                     uint64_t gbase, lu8 *kbuf) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t ko = (uint32_t)(kb0 & 15);
    if (!sequential) {
        const uint32_t R = v.count;
        uint64_t ecarry = ent0, kcarry = kb0;
        for (uint32_t q0 = 0; q0 < R; q0 += 64) {
            const uint32_t q = q0 + l;
            uint32_t pos = 0, end = 0, ne = 0, nk = 0;
            bool exact = true;
            if constexpr (std::is_same<P, const lu8 *>::value) {
                // header-only steps (single-byte varints, no timestamps), flags checked off the chain;
                // any other shape in the batch: the exact walk below
                bool ok = true;
                if (q < R) {
                    pos = (uint32_t)rd_be(v.offs + 2 * q, 2);
                    end = (q + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * q + 2, 2) : v.data_end;
                    uint32_t p = pos, fl = 0, bad = 0;
                    while (p < end) {
                        const uint32_t h = lds_read4(v.d + p);
                        bad |= (fl & (SDB_FLAG_HAS_EXPIRE_TS | SDB_FLAG_HAS_CREATE_TS)) ? 1u : 0u;
                        const uint32_t un = (h >> 8) & 0xFF, vl = (h >> 16) & 0xFF;
                        if ((h & 0x808080u) || p + 12 + un + vl > end) {
                            ok = false;
                            break;
                        }
                        fl = v.d[p + 11 + un + vl];
                        if (kbuf && q < 4 && ne < 32) ((lu16 *)(kbuf + kRowTmp))[q * 32 + ne] = (uint16_t)p;
                        ne++;
                        nk += (h & 0xFF) + un;
                        p += 12 + un + vl;
                    }
                    bad |= (fl & (SDB_FLAG_HAS_EXPIRE_TS | SDB_FLAG_HAS_CREATE_TS)) ? 1u : 0u;
                    if (p != end || bad) ok = false;
                }
                exact = __ballot(!ok) != 0;
                if (exact) ne = nk = 0;
            }
            if (exact && q < R) {
                pos = (uint32_t)rd_be(v.offs + 2 * q, 2);
                end = (q + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * q + 2, 2) : v.data_end;
                uint32_t p = pos;
                while (p < end) {
                    RowV2 r;
                    parse_v2(v.d, v.data_end, p, &r);
                    ne++;
                    nk += r.shared + r.unshared;
                    p = r.next;
                }
            }
            const uint64_t ie = wave_incl_scan((uint64_t)ne), ik = wave_incl_scan((uint64_t)nk);
            uint64_t idx = ecarry + ie - ne, kp = kcarry + ik - nk;
            bool done_fast = false;
            if constexpr (std::is_same<P, const lu8 *>::value) {
                // lane = row: the block has the fast shape, <= 4 regions of <= 32 rows, <= 64 rows, keys of
                // <= 16 bytes, and walk 1 recorded every row's position; the rows are parsed in parallel
                // and key byte b of row j is suffix byte b of the last row r <= j with shared_r <= b (a
                // max-scan over the lanes per byte position)
                const uint32_t NE = (uint32_t)wave_readlane(ie, 63);
                const uint32_t maxne = wave_max(q < R ? ne : 0u);
                const uint64_t kbn_blk = wave_readlane(ik, 63);
                if (!exact && kbuf && q0 == 0 && R <= 4 && NE <= 64 && maxne <= 32 && kbn_blk + 16 <= kRowTmp) {
                    const uint32_t j = l;
                    const bool live = j < NE;
                    const uint32_t exn = (uint32_t)(ie - ne);  // region lane: its first row
                    uint32_t qj = 0;
#pragma unroll
                    for (uint32_t qq = 1; qq < 4; qq++)
                        if (qq < R && j >= (uint32_t)__builtin_amdgcn_readlane((int)exn, (int)qq)) qj = qq;
                    const uint32_t b0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(qj << 2), (int)exn);
                    const uint32_t pj = live ? (uint32_t)((const lu16 *)(kbuf + kRowTmp))[qj * 32 + (j - b0)] : 0;
                    const uint32_t h = lds_read4(v.d + pj);
                    const uint32_t sh = live ? (h & 0xFF) : 0, un = live ? (h >> 8) & 0xFF : 0, vl = (h >> 16) & 0xFF;
                    uint32_t x[4];
                    lds_read16(v.d + pj + 3 + un + vl, x);
                    const uint32_t klen = sh + un;
                    if (wave_max(klen) <= 16) {
                        const uint32_t kinc = wave_incl_scan(klen);
                        const uint32_t krel = kinc - klen;  // key position of row j in the block's keys
                        const uint32_t baddr = pj + 3 - sh;  // key byte b of row j (b >= sh) is v.d[baddr + b]
                        lu8 *dst = kbuf + ko + krel;
#pragma unroll
                        for (uint32_t b = 0; b < 16; b++) {
                            const uint32_t m = (live && sh <= b) ? j : 0;
                            const uint32_t src = wave_incl_scan_op(m, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
                            const uint32_t sa = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)baddr);
                            if (b < klen) dst[b] = v.d[sa + b];
                        }
                        if (live) {
                            if (a.descending) key_store_desc(a, kb0 + krel, dst, klen);
                            const uint8_t f = (uint8_t)x[2];
                            put_entry(a, ecarry + j, kb0 + krel, klen, gbase + (pj + 3 + un),
                                      (f & SDB_FLAG_TOMBSTONE) ? 0 : vl, be64_at(x[0], x[1]), f, 0, 0);
                        }
                        done_fast = true;
                    }
                }
                if (!done_fast && !exact && kbuf) {
                    // the batch has the fast shape (checked by the counting walk): header-only steps; the
                    // trailer, the previous key and the suffix are 16-byte windows off the chain, and
                    // keys of <= 16 bytes are merged in registers and written byte by byte (no waits)
                    done_fast = true;
                    if (q < R) {
                        uint64_t prev_kp = 0;
                        uint32_t p = pos;
                        while (p < end) {
                            const uint32_t h = lds_read4(v.d + p);
                            const uint32_t sh = h & 0xFF, un = (h >> 8) & 0xFF, vl = (h >> 16) & 0xFF;
                            const uint32_t t = p + 3 + un + vl;
                            uint32_t x[4];
                            lds_read16(v.d + t, x);
                            const uint32_t klen = sh + un;
                            lu8 *dst = kbuf + ko + (uint32_t)(kp - kb0);
                            if (klen <= 16) {
                                uint32_t pw[4] = {0, 0, 0, 0}, sw[4];
                                if (sh) lds_read16(kbuf + ko + (uint32_t)(prev_kp - kb0), pw);
                                lds_read16(v.d + p + 3, sw);
                                uint64_t lo = (uint64_t)pw[0] | ((uint64_t)pw[1] << 32), hi = (uint64_t)pw[2] | ((uint64_t)pw[3] << 32);
                                key16_merge(lo, hi, sh, sw);
#pragma unroll
                                for (uint32_t b = 0; b < 16; b++)
                                    if (b < klen) dst[b] = (uint8_t)(b < 8 ? lo >> (8 * b) : hi >> (8 * (b - 8)));
                            } else {
                                lds_copy_small(dst, kbuf + ko + (uint32_t)(prev_kp - kb0), sh);
                                for (uint32_t b = 0; b < un; b++) dst[sh + b] = v.d[p + 3 + b];
                            }
                            if (a.descending) key_store_desc(a, kp, dst, klen);
                            const uint8_t f = (uint8_t)x[2];
                            put_entry(a, idx, kp, klen, gbase + (p + 3 + un), (f & SDB_FLAG_TOMBSTONE) ? 0 : vl,
                                      be64_at(x[0], x[1]), f, 0, 0);
                            prev_kp = kp;
                            kp += klen;
                            idx++;
                            p = t + 9;
                        }
                    }
                }
            }
            if (!done_fast && q < R) {
                uint64_t prev_kp = 0;
                uint32_t prev_kl = 0;
                uint32_t p = pos;
                while (p < end) {
                    RowV2 r;
                    parse_v2(v.d, v.data_end, p, &r);
                    const uint32_t kl = r.shared + r.unshared;
                    if (kbuf) {
                        lu8 *dst = kbuf + ko + (uint32_t)(kp - kb0);
                        lds_copy_small(dst, kbuf + ko + (uint32_t)(prev_kp - kb0), r.shared);
                        for (uint32_t x = 0; x < r.unshared; x++) dst[r.shared + x] = v.d[r.suf_pos + x];
                        if (a.descending) key_store_desc(a, kp, dst, kl);
                    } else {
                        uint8_t *dst = key_dst(a, kp, kl);
                        const uint8_t *pk = key_dst(a, prev_kp, prev_kl);
                        for (uint32_t x = 0; x < r.shared; x++) dst[x] = pk[x];
                        for (uint32_t x = 0; x < r.unshared; x++) dst[r.shared + x] = v.d[r.suf_pos + x];
                    }
                    const uint32_t vl = (r.flags & SDB_FLAG_TOMBSTONE) ? 0 : r.vlen;
                    put_entry(a, idx, kp, kl, gbase + r.val_pos, vl, r.seq, r.flags, r.cts, r.ets);
                    prev_kp = kp;
                    prev_kl = kl;
                    kp += kl;
                    idx++;
                    p = r.next;
                }
            }
            ecarry += wave_readlane(ie, 63);
            kcarry += wave_readlane(ik, 63);
        }
    } else if (l == 0) {
        // sequential walk (BlockIteratorV2 ascending); the initial current_key is the key at restart 0
        uint64_t idx = ent0, kp = kb0, prev_kp = 0;
        uint32_t pos = 0, prev_kl = 0;
        uint32_t p0 = (uint32_t)rd_be(v.offs, 2), sh = 0, un = 0, vl0 = 0;
        rd_varint(v.d, v.data_end, &p0, &sh);
        rd_varint(v.d, v.data_end, &p0, &un);
        rd_varint(v.d, v.data_end, &p0, &vl0);
        const uint32_t init_key = p0;  // position of restart 0's key suffix (= its whole key)
        bool first = true;
        while (pos < v.data_end) {
            RowV2 r;
            parse_v2(v.d, v.data_end, pos, &r);
            const uint32_t kl = r.shared + r.unshared;
            if (kbuf) {
                lu8 *dst = kbuf + ko + (uint32_t)(kp - kb0);
                for (uint32_t x = 0; x < r.shared; x++) dst[x] = first ? v.d[init_key + x] : kbuf[ko + (uint32_t)(prev_kp - kb0) + x];
                for (uint32_t x = 0; x < r.unshared; x++) dst[r.shared + x] = v.d[r.suf_pos + x];
                if (a.descending) key_store_desc(a, kp, dst, kl);
            } else {
                uint8_t *dst = key_dst(a, kp, kl);
                const uint8_t *pk = key_dst(a, prev_kp, prev_kl);
                for (uint32_t x = 0; x < r.shared; x++) dst[x] = first ? v.d[init_key + x] : pk[x];
                for (uint32_t x = 0; x < r.unshared; x++) dst[r.shared + x] = v.d[r.suf_pos + x];
            }
            const uint32_t vl = (r.flags & SDB_FLAG_TOMBSTONE) ? 0 : r.vlen;
            put_entry(a, idx, kp, kl, gbase + r.val_pos, vl, r.seq, r.flags, r.cts, r.ets);
            prev_kp = kp;
            prev_kl = kl;
            kp += kl;
            idx++;
            first = false;
            pos = r.next;
        }
    }
}

// V2 emit, lane = row, for blocks whose row positions the count pass recorded (rc: rows of restart
// regions 0..3, 16 bits each; pos: 4 x 32 positions): no walk at all.  Key byte b of row j is suffix byte
// b of the last row r <= j with shared_r <= b (a max-scan over the lanes per byte position).
SDB_DEV void emit_v2_rows(const DecodeArgs &a, const LdsBlockView &v, uint64_t rc, const lu16 *pos, uint64_t ent0,
                          uint64_t kb0, uint64_t gbase, lu8 *kbuf) {
    const uint32_t j = (uint32_t)lane_id();
    const uint32_t c0 = rc & 0xFFFF, c1 = (rc >> 16) & 0xFFFF, c2 = (rc >> 32) & 0xFFFF, c3 = (rc >> 48) & 0xFFFF;
    const uint32_t NE = c0 + c1 + c2 + c3;
    const bool live = j < NE;
    uint32_t q = 0, i = j;
    if (i >= c0) { i -= c0; q = 1; }
    if (q == 1 && i >= c1) { i -= c1; q = 2; }
    if (q == 2 && i >= c2) { i -= c2; q = 3; }
    const uint32_t pj = live ? pos[q * 32 + i] : 0;
    const uint32_t h = lds_read4(v.d + pj);
    const uint32_t sh = live ? (h & 0xFF) : 0, un = live ? (h >> 8) & 0xFF : 0, vl = (h >> 16) & 0xFF;
    uint32_t x[4];
    lds_read16(v.d + pj + 3 + un + vl, x);
    const uint32_t klen = sh + un;
    const uint32_t kinc = wave_incl_scan(klen);
    const uint32_t krel = kinc - klen;   // key position of row j among the block's keys
    const uint32_t baddr = pj + 3 - sh;  // key byte b of row j (b >= sh) is v.d[baddr + b]
    lu8 *dst = kbuf + (uint32_t)(kb0 & 15) + krel;
#pragma unroll
    for (uint32_t b = 0; b < 16; b++) {
        const uint32_t m = (live && sh <= b) ? j : 0;
        const uint32_t src = wave_incl_scan_op(m, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
        const uint32_t sa = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)baddr);
        if (b < klen) dst[b] = v.d[sa + b];
    }
    if (live) {
        if (a.descending) key_store_desc(a, kb0 + krel, dst, klen);
        const uint8_t f = (uint8_t)x[2];
        put_entry(a, ent0 + j, kb0 + krel, klen, gbase + (pj + 3 + un), (f & SDB_FLAG_TOMBSTONE) ? 0 : vl,
                  be64_at(x[0], x[1]), f, 0, 0);
    }
}

// V1 emit (BlockIterator, block_iterator.rs:54-267): lane = entry, key = first key's prefix + suffix.
template <typename P>
SDB_DEV void emit_v1(const DecodeArgs &a, const BlockViewT<P> &v, uint64_t ent0, uint64_t kb0, uint64_t gbase) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t R = v.count;
    uint64_t carry = kb0;
    for (uint32_t g0 = 0; g0 < R; g0 += 64) {
        const uint32_t i = g0 + l;
        RowV0 r;
        uint32_t kl = 0;
        if (i < R) {
            parse_v0(v.d, v.data_end, (uint32_t)rd_be(v.offs + 2 * i, 2), &r);
            kl = r.prefix + r.suf;
        }
        const uint64_t inc = wave_incl_scan((uint64_t)kl);
        if (i < R) {
            const uint64_t kp = carry + inc - kl;
            uint8_t *dst = key_dst(a, kp, kl);
            for (uint32_t q = 0; q < r.prefix; q++) dst[q] = v.d[4 + q];
            for (uint32_t q = 0; q < r.suf; q++) dst[r.prefix + q] = v.d[r.suf_pos + q];
            put_entry(a, ent0 + i, kp, kl, gbase + r.val_pos, r.vlen, r.seq, r.flags, r.cts, r.ets);
        }
        carry += wave_readlane(inc, 63);
    }
}

// Emit pass of a regular big V2 block by pieces (the count pass accepted it as regular): keys restored
// in LDS when a piece's keys fit, else straight into the arena.
SDB_DEV bool emit_v2_pieces(const DecodeArgs &a, uint64_t s, const BlockView &v, lu8 *img, lu8 *kbuf, uint64_t ent0,
                            uint64_t kb0) {
    uint64_t ent = ent0, kb = kb0;
    return for_each_piece(a, s, v, img, [&](const LdsBlockView &pv, uint32_t base) {
        // as a small block: the walks record the row positions of <= 4 regions in kbuf's row table, and
        // the lane-per-row emit parses from them
        lu16 *rows = (lu16 *)(kbuf + kRowTmp);
        Tally pt{0, 0, 0, false};
        uint64_t rc = ~0ull;
#ifndef SDB_PIECE_ROWS
#define SDB_PIECE_ROWS 1
#endif
        if (!SDB_PIECE_ROWS || (!tally_v2_spec(pv, pt, (uint16_t *)rows, &rc) && !tally_v2_fast(pv, pt, (uint16_t *)rows, &rc))) {
            pt = tally_v2(pv);
            rc = ~0ull;
        }
        rc = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)rc) |
             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(rc >> 32)) << 32);  // lane 0 wrote it
        const bool lds_keys = pt.key_bytes + 16 <= kDecKeys;
        if (rc != ~0ull && pt.key_bytes + 16 <= kRowTmp) {
            wave_sync_d();
            emit_v2_rows(a, pv, rc, rows, ent, kb, s + base, kbuf);
        } else {
            emit_v2(a, pv, false, ent, kb, s + base, lds_keys ? kbuf : nullptr);
        }
        if (lds_keys && !a.descending) {  // (descending: each lane stored its keys)
            wave_sync_d();
            wave_store_bytes(a.out.key_arena + kb, kbuf, pt.key_bytes);
        }
        ent += pt.entries;
        kb += pt.key_bytes;
        return true;
    });
}

SDB_DEV void dec_finish(const DecodeArgs &a) {
    sdb_decode_summary *s = a.out.summary;
    const uint64_t ne = a.ent_start[a.nblocks], kb = a.key_start[a.nblocks];
    s->num_entries = ne;
    s->key_bytes = kb;
    s->num_bad_blocks = atomicAdd(a.nbad, 0ull);
    const unsigned long long e = atomicOr(a.err, 0ull);
    s->status = e == ~0ull ? 0 : (int32_t)(e & 0xFF);
    s->pad = 0;
    a.out.block_entry_start[a.nblocks] = ne;
    // over capacity nothing was written; fail-fast still reports a bad block's error first (read_blocks fails
    // on the block; k_dec_emit checked the deferred checksums without emitting)
    if (ne > a.out.cap_entries || kb > a.out.key_arena_cap) s->status = (a.fail_fast && e != ~0ull) ? s->status : SDB_INVALID_ARGUMENT;
    else a.out.key_off[ne] = kb;
}

// D3 emit: one wave per block, stage again (no CRC: the count pass checked it), write the columns.
// k_dec_emit takes the blocks the count pass left unflagged (V2, one wave image, row positions recorded:
// the lane-per-row emit) and writes every block's entry start; k_dec_emit_gen the kFlagGen blocks (V1,
// sequential or unrecorded walks, blocks over one image), so the common path carries none of their
// registers.  Small batches (a.small: <= 1024 blocks, one per wave — a 2 MiB read_blocks range is ~520)
// skip the three scan kernels: every workgroup of k_dec_emit scans the per-block counts itself (one
// 1024-thread scan, workgroup 0 stores the result for k_dec_emit_gen), and the last workgroup of
// k_dec_emit_gen writes the summary (no k_dec_finish launch).
// DESC: the order as a compile-time constant of the local copy, so the ascending instance carries none
// of the mirroring
#ifndef SDB_DEC_EMIT_REV
#define SDB_DEC_EMIT_REV 1
#endif
constexpr bool kEmitRev = SDB_DEC_EMIT_REV != 0;

template <bool DESC>
__global__ __launch_bounds__(kEmThreads) __attribute__((amdgpu_waves_per_eu(kEmEu))) void k_dec_emit(DecodeArgs a0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    DecodeArgs a = a0;  // + the output totals (descending order mirrors every entry and key against them)
    a.descending = DESC ? 1u : 0u;
    bool run = true;
    uint64_t s_ent0 = 0, s_ent1 = 0, s_kb0 = 0, s_kb1 = 0, tot_ent = 0, tot_kb = 0;
    if (a.small) {
        // exclusive scans of cnt / kbytes over all blocks; scratch in wave 0's (still unused) region
        uint64_t *sw = (uint64_t *)smem;
        uint64_t *sres = sw + 32;
        const uint32_t t = threadIdx.x, b0 = blockIdx.x * (kEmThreads / 64);
        const uint64_t vx = t < a.nblocks ? a.cnt[t] : 0, vy = t < a.nblocks ? a.kbytes[t] : 0;
        const uint64_t ex = block_excl_scan_u64(vx, sw, &tot_ent);
        const uint64_t ey = block_excl_scan_u64(vy, sw, &tot_kb);
        if (t >= b0 && t < b0 + kEmThreads / 64) {
            uint64_t *r = sres + 4 * (t - b0);
            r[0] = ex;
            r[1] = ex + vx;
            r[2] = ey;
            r[3] = ey + vy;
        }
        if (blockIdx.x == 0 && t < a.nblocks) {
            a.ent_start[t] = ex;
            a.key_start[t] = ey;
        }
        if (blockIdx.x == 0 && t == 0) {  // nblocks may be 1024 = blockDim.x
            a.ent_start[a.nblocks] = tot_ent;
            a.key_start[a.nblocks] = tot_kb;
        }
        __syncthreads();
        const uint64_t *r = sres + 4 * (threadIdx.x >> 6);
        auto uni = [](uint64_t v) {  // wave-uniform: keep it in scalar registers
            return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
        };
        s_ent0 = uni(r[0]);
        s_ent1 = uni(r[1]);
        s_kb0 = uni(r[2]);
        s_kb1 = uni(r[3]);
        __syncthreads();
    } else {
        tot_ent = a.ent_start[a.nblocks];
        tot_kb = a.key_start[a.nblocks];
    }
    const uint32_t wave = threadIdx.x >> 6;
    const int l = lane_id();
    lu8 *img = (lu8 *)smem + kDecTabLds + wave * kDecWaveLds + kDecGuard;
    lu8 *kbuf = img + kDecImg;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    (void)gwave;
    const bool ff = a.fail_fast != 0;
    if (ff) {  // fail-fast: this pass verifies the checksums (tables at LDS address 0, zero guards)
        if (lds_addr((const void *)smem) != 0) {
            if (threadIdx.x == 0) atomicMin(a.err, (unsigned long long)SDB_DEVICE_ERROR);
            return;
        }
        dec_crc_tables_to_lds((lu32 *)smem);
        if (l < kDecGuard / 4) ((lu32 *)(img - kDecGuard))[l] = 0;
        __syncthreads();
    }
    // capacity guard: if the counted output does not fit the caller's arrays, write nothing (fail-fast still
    // walks the blocks to verify the checksums the count pass deferred: a corrupt block whose garbage
    // raises the counts must report CHECKSUM_MISMATCH, not the capacity)
    if (tot_ent > a.out.cap_entries || tot_kb > a.out.key_arena_cap) run = false;
    a.dn = tot_ent;
    a.dkb = tot_kb;
    // Software pipeline (as k_dec_count): block k's granules, scan results / flag / row count and row
    // positions landed; block k + nwaves's granules, metadata and row positions in flight, with the
    // offsets of block k + 2 nwaves.  The metadata come in ONE vector load (lane j: 32-bit word j of
    // the block's scan results, row count, flag word and the offsets two blocks ahead), every load is
    // unconditional (clamped block indices), so the compiler's only vmcnt waits are the hand-overs.
    if (!(run || ff) || gwave >= a.nblocks) return;
    const bool small = a.small != 0;
    const uint64_t lastk = a.nblocks - 1;
    auto clampk = [&](uint64_t x) { return x < a.nblocks ? x : lastk; };
    auto gather = [&](uint64_t kn, uint64_t k2) -> uint32_t {
        const uint32_t *p = (const uint32_t *)(a.block_off + k2);  // lanes 11, 12 (and lanes >= 15: unused)
        if (l < 4) p = (const uint32_t *)(a.ent_start + kn) + l;
        else if (l < 8) p = (const uint32_t *)(a.key_start + kn) + (l - 4);
        else if (l < 10) p = (const uint32_t *)(a.rcnt + kn) + (l - 8);
        else if (l == 10) p = (const uint32_t *)(a.flag + (kn & ~3ull));  // 256-byte aligned array
        else if (l == 12) p = (const uint32_t *)(a.block_off + k2) + 1;
        else if (l == 13 || l == 14)
            p = (const uint32_t *)(a.block_end ? a.block_end + k2 : a.block_off + k2 + 1) + (l - 13);
        return *p;
    };
    auto u64_at = [](uint32_t g, int lane) {
        return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)g, lane) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)g, lane + 1) << 32);
    };
    auto rowpos_load = [&](uint64_t kk) -> uint32_t { return ((const uint32_t *)(a.rowpos + 128 * kk))[l]; };
    // wave step k takes block B(k): descending block order when SDB_DEC_EMIT_REV, so the emit starts on the
    // blocks the count pass read last (still in the Infinity Cache)
    const bool rev = kEmitRev && !small;  // (small: each wave's scan results above are for block gwave)
    auto B = [&](uint64_t x) -> uint64_t { return rev ? lastk - x : x; };
    uint64_t k = gwave, kb = B(k);
    uint64_t s = a.block_off[kb], e = block_end_of(a, kb);
    uint32_t gcur = gather(kb, B(clampk(k + nwaves)));
    uint32_t rp = rowpos_load(kb);
    Granules cur;
    gran_load_u(a, s, e, cur);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the pipeline starts with nothing in flight
    uint64_t s1 = u64_at(gcur, 11), e1 = u64_at(gcur, 13);
    for (;;) {
        // block k's granules -> its LDS image first, so their registers take the next block's
        if (dec_fast(s, e)) gran_store(s, e, cur, img);
        const uint64_t kn = B(clampk(k + nwaves)), k2 = B(clampk(k + 2 * nwaves));
        gran_load_u(a, s1, e1, cur);
        const uint32_t gnx = gather(kn, k2);
        const uint32_t rpn = rowpos_load(kn);
        do {
            const uint64_t ent0 = small ? s_ent0 : u64_at(gcur, 0), ent1 = small ? s_ent1 : u64_at(gcur, 2);
            const uint64_t kb0 = small ? s_kb0 : u64_at(gcur, 4), kb1 = small ? s_kb1 : u64_at(gcur, 6);
            const uint64_t rcw = u64_at(gcur, 8);
            const uint32_t fw = (uint32_t)__builtin_amdgcn_readlane((int)gcur, 10);
            if (run && l == 0) a.out.block_entry_start[kb] = ent0;
            const uint32_t fb = (fw >> (8 * (kb & 3))) & 0xFF;
            const bool skip = ent1 == ent0 || (fb & kFlagGen);  // nothing to emit, or k_dec_emit_gen's
            // fail-fast: every block of one wave image the count pass did not reject is checked here
            if ((skip || !run) && !(ff && !(fb & kFlagBad) && dec_fast(s, e))) break;
            DEC_T(t0);
            const LdsBlockView v = stage_lds(a, s, e, img, ff, nullptr, true);
            if (v.status) {  // fail-fast: a checksum mismatch (the count pass accepted the rest)
                if (l == 0) {
                    atomicMin(a.err, (unsigned long long)((kb << 8) | (uint64_t)v.status));
                    const unsigned long long slot = atomicAdd(a.nbad, 1ull);
                    if (slot < a.bad_cap) a.bad_block[slot] = (uint32_t)kb;
                }
                break;
            }
            if (skip || !run) break;
            DEC_T(t1);
            ((lu32 *)(kbuf + kRowTmp))[l] = rp;
            wave_sync_d();
            emit_v2_rows(a, v, rcw, (const lu16 *)(kbuf + kRowTmp), ent0, kb0, s, kbuf);
            DEC_T(t2);
            if (!a.descending) {  // (descending: each lane stored its keys)
                wave_sync_d();
                wave_store_bytes(a.out.key_arena + kb0, kbuf, kb1 - kb0);
            }
            DEC_T(t3);
            DEC_ACC(1, 0, t1 - t0);
            DEC_ACC(1, 1, t2 - t1);
            DEC_ACC(1, 2, t3 - t2);
            DEC_ACC(1, 3, 1);
        } while (false);
        wave_sync_d();
        k += nwaves;
        if (k >= a.nblocks) break;
        kb = B(k);
        gcur = gnx;
        rp = rpn;
        s = s1;
        e = e1;
        s1 = u64_at(gnx, 11);
        e1 = u64_at(gnx, 13);
    }
}

// D3 emit of the kFlagGen blocks: V1 rows, V2 blocks walked sequentially or by regions without recorded
// rows, keys over the row table, and blocks over one wave image (restart-region pieces, or the walk from
// HBM).  Small batches: the last workgroup writes the summary.
template <bool DESC>
__global__ __launch_bounds__(kEmThreads) __attribute__((amdgpu_waves_per_eu(kEmEu))) void k_dec_emit_gen(DecodeArgs a0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    DecodeArgs a = a0;
    a.descending = DESC ? 1u : 0u;
    const uint64_t tot_ent = a.ent_start[a.nblocks], tot_kb = a.key_start[a.nblocks];
    const bool run = tot_ent <= a.out.cap_entries && tot_kb <= a.out.key_arena_cap;
    a.dn = tot_ent;
    a.dkb = tot_kb;
    const uint32_t wave = threadIdx.x >> 6;
    const int l = lane_id();
    lu8 *img = (lu8 *)smem + kDecTabLds + wave * kDecWaveLds + kDecGuard;
    lu8 *kbuf = img + kDecImg;
    uint8_t *stage = (uint8_t *)img;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (run && wg_any_flagged(a, kFlagGen, (uint32_t *)smem)) for_flagged(a, kFlagGen, gwave, nwaves, [&](uint64_t k) {
        const uint64_t ent0 = a.ent_start[k], kb0 = a.key_start[k];
        const uint64_t kbn = a.key_start[k + 1] - kb0;
        if (a.ent_start[k + 1] == ent0) return;
        const uint8_t f = a.flag[k];
        const bool seq = (f & kFlagSeq) != 0;
        const uint64_t s = a.block_off[k], e = block_end_of(a, k);
        if (dec_fast(s, e)) {
            const LdsBlockView v = stage_lds(a, s, e, img, false, nullptr);
            if (v.status) return;
            if (a.version == 1) {
                emit_v1(a, v, ent0, kb0, s);
            } else {
                const bool lds_keys = kbn + 16 <= kDecKeys;
                const uint64_t rc = seq ? ~0ull : a.rcnt[k];
                if (rc != ~0ull && kbn + 16 <= kRowTmp) {
                    ((lu32 *)(kbuf + kRowTmp))[l] = ((const uint32_t *)(a.rowpos + 128 * k))[l];
                    wave_sync_d();
                    emit_v2_rows(a, v, rc, (const lu16 *)(kbuf + kRowTmp), ent0, kb0, s, kbuf);
                } else {
                    emit_v2(a, v, seq, ent0, kb0, s, lds_keys ? kbuf : nullptr);
                }
                if (lds_keys && !a.descending) {
                    wave_sync_d();
                    wave_store_bytes(a.out.key_arena + kb0, kbuf, kbn);
                }
            }
        } else {
            const BlockView v = load_block(a, k, stage, nullptr, kDecCap, false);
            if (v.status) return;
            if (a.version == 1) emit_v1(a, v, ent0, kb0, s);
            else if (seq || !emit_v2_pieces(a, s, v, img, kbuf, ent0, kb0)) emit_v2(a, v, seq, ent0, kb0, s, nullptr);
        }
        wave_sync_d();
    });
    if (a.small) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
                __threadfence();
                dec_finish(a);
            }
        }
    }
}

// --- scans ------------------------------------------------------------------------------------------
constexpr uint32_t kScanTile = 1024;

__global__ __launch_bounds__(1024) void k_scan_tiles(const uint64_t *x, const uint64_t *y, uint64_t n,
                                                     uint64_t *tx, uint64_t *ty) {
    __shared__ uint64_t s_w[17];
    uint64_t i = (uint64_t)blockIdx.x * kScanTile + threadIdx.x;
    uint64_t vx = i < n ? x[i] : 0, vy = i < n ? y[i] : 0;
    uint64_t sx, sy;
    block_excl_scan_u64(vx, s_w, &sx);
    block_excl_scan_u64(vy, s_w, &sy);
    if (threadIdx.x == 0) {
        tx[blockIdx.x] = sx;
        ty[blockIdx.x] = sy;
    }
}

__global__ __launch_bounds__(1024) void k_scan_top(uint64_t *tx, uint64_t *ty, uint64_t nt) {
    __shared__ uint64_t s_w[17];
    uint64_t cx = 0, cy = 0;
    for (uint64_t b = 0; b < nt; b += kScanTile) {
        uint64_t i = b + threadIdx.x;
        uint64_t vx = i < nt ? tx[i] : 0, vy = i < nt ? ty[i] : 0;
        uint64_t sx, sy;
        uint64_t ex = block_excl_scan_u64(vx, s_w, &sx);
        uint64_t ey = block_excl_scan_u64(vy, s_w, &sy);
        if (i < nt) {
            tx[i] = cx + ex;
            ty[i] = cy + ey;
        }
        cx += sx;
        cy += sy;
    }
    if (threadIdx.x == 0) {
        tx[nt] = cx;
        ty[nt] = cy;
    }
}

__global__ __launch_bounds__(1024) void k_scan_apply(const uint64_t *x, const uint64_t *y, uint64_t n,
                                                     const uint64_t *tx, const uint64_t *ty, uint64_t nt,
                                                     uint64_t *ox, uint64_t *oy) {
    __shared__ uint64_t s_w[17];
    uint64_t i = (uint64_t)blockIdx.x * kScanTile + threadIdx.x;
    uint64_t vx = i < n ? x[i] : 0, vy = i < n ? y[i] : 0;
    uint64_t sx, sy;
    uint64_t ex = block_excl_scan_u64(vx, s_w, &sx);
    uint64_t ey = block_excl_scan_u64(vy, s_w, &sy);
    if (i < n) {
        ox[i] = tx[blockIdx.x] + ex;
        oy[i] = ty[blockIdx.x] + ey;
    }
    if (i == n - 1) {
        ox[n] = tx[nt];
        oy[n] = ty[nt];
    }
}

// Exclusive scans of x and y over n values (ox/oy: n + 1 values, the totals last); tx/ty: (n + 1023) /
// 1024 + 1 tile sums each.  Shared with the decompression plan (sdb_codec.hip).
hipError_t launch_excl_scan2(const uint64_t *x, const uint64_t *y, uint64_t n, uint64_t *tx, uint64_t *ty,
                             uint64_t *ox, uint64_t *oy, hipStream_t st) {
    if (n == 0) {
        hipError_t e = hipMemsetAsync(ox, 0, 8, st);
        return e != hipSuccess ? e : hipMemsetAsync(oy, 0, 8, st);
    }
    const uint64_t nt = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)nt), dim3(kScanTile), 0, st, x, y, n, tx, ty);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanTile), 0, st, tx, ty, nt);
    hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nt), dim3(kScanTile), 0, st, x, y, n, tx, ty, nt, ox, oy);
    return hipGetLastError();
}

__global__ void k_dec_init(DecodeArgs a) {
    if (threadIdx.x == 0) {
        *a.err = ~0ull;
        *a.nbad = 0;
        *a.done = 0;
    }
}

__global__ void k_dec_finish(DecodeArgs a) {
    if (threadIdx.x == 0) dec_finish(a);
}

hipError_t launch_decode(DecodeArgs a, hipStream_t st) {
    static std::once_flag attrs;
    static hipError_t attr_err = hipSuccess;
    std::call_once(attrs, [] {
        attr_err = hipFuncSetAttribute((const void *)k_dec_count, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kCntLds);
        if (attr_err == hipSuccess)
            attr_err = hipFuncSetAttribute((const void *)k_dec_count_big, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)kCntLds);
        for (const void *f : {(const void *)k_dec_emit<false>, (const void *)k_dec_emit<true>,
                              (const void *)k_dec_emit_gen<false>, (const void *)k_dec_emit_gen<true>})
            if (attr_err == hipSuccess)
                attr_err = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDecLds);
    });
    if (attr_err != hipSuccess) return attr_err;
    hipLaunchKernelGGL(k_dec_init, dim3(1), dim3(64), 0, st, a);
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    auto grid = [&](uint32_t threads, uint32_t per_cu) {  // one wave per block, at most per_cu workgroups per CU
        uint64_t g = (a.nblocks + threads / 64 - 1) / (threads / 64);
        if (cus > 0 && g > (uint64_t)cus * per_cu) g = (uint64_t)cus * per_cu;
        return g ? g : 1;
    };
    const uint64_t wgc = grid(kCntThreads, kCntWg), wgs = grid(kEmThreads, kEmWg);
    const size_t lds = kDecLds;
    if (a.nblocks) {
        hipLaunchKernelGGL(k_dec_count, dim3((uint32_t)wgc), dim3(kCntThreads), kCntLds, st, a);
        hipLaunchKernelGGL(k_dec_count_big, dim3((uint32_t)wgc), dim3(kCntThreads), kCntLds, st, a);
    }
    // scans: ent_start = excl(cnt), key_start = excl(kbytes); small batches scan inside k_dec_emit
    a.small = a.nblocks > 0 && a.nblocks <= kEmThreads && wgs * (kEmThreads / 64) >= a.nblocks ? 1u : 0u;
    uint64_t nt = (a.nblocks + kScanTile - 1) / kScanTile;
    if (a.small) {
    } else if (a.nblocks) {
        hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)nt), dim3(kScanTile), 0, st, a.cnt, a.kbytes, a.nblocks,
                           a.tile_x, a.tile_y);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanTile), 0, st, a.tile_x, a.tile_y, nt);
        hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nt), dim3(kScanTile), 0, st, a.cnt, a.kbytes, a.nblocks,
                           a.tile_x, a.tile_y, nt, a.ent_start, a.key_start);
    } else {
        hipMemsetAsync(a.ent_start, 0, 8, st);
        hipMemsetAsync(a.key_start, 0, 8, st);
    }
    if (a.nblocks) {
        if (a.descending) {
            hipLaunchKernelGGL(k_dec_emit<true>, dim3((uint32_t)wgs), dim3(kEmThreads), lds, st, a);
            hipLaunchKernelGGL(k_dec_emit_gen<true>, dim3((uint32_t)wgs), dim3(kEmThreads), lds, st, a);
        } else {
            hipLaunchKernelGGL(k_dec_emit<false>, dim3((uint32_t)wgs), dim3(kEmThreads), lds, st, a);
            hipLaunchKernelGGL(k_dec_emit_gen<false>, dim3((uint32_t)wgs), dim3(kEmThreads), lds, st, a);
        }
    }
    if (!a.small) hipLaunchKernelGGL(k_dec_finish, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace sdb

#ifdef SDB_PHASE_TIMING
extern "C" int sdb_diag_dec_phase(uint64_t *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sdb::g_dec_phase), sizeof(uint64_t) * 2 * 8192 * 4) == hipSuccess ? 0 : -1;
}
#endif
