// sdb_codec_enc.hip — the compressing write side of SURVEY §8(f) row f3 for gfx950.
//
// Replaces compress_and_transform (slatedb/src/format/sst.rs:525-554) with SsTableFormat::compress
// (format/sst.rs:557-594) for every block of an encoded data section: the codec's bytes of
// Block::encode(), then the CRC32 (BE) of those compressed bytes:
//   Lz4    lz4_flex 0.11.6 block::compress_prepend_size: u32 LE length ++ one LZ4 block;
//   Snappy snap 1.1.1 raw::Encoder::compress_vec: varint length ++ Snappy raw elements;
//   Zlib   flate2 1.1.9 ZlibEncoder (default level 6): 78 9C ++ deflate ++ Adler-32 BE;
//   Zstd   zstd 0.13.3 bulk::compress(data, 3): one frame with Frame_Content_Size (single segment).
// A compressor's output bytes are a choice of its match finder and entropy coder, not of the format:
// these streams are valid for the formats (they decode through the reference's decompressors — and
// sdb_decompress_blocks, the oracle, pyarrow / zlib in the tests — to the same block bytes) and compress
// to within a few per cent of the canonical libraries, but they are not the crates' bytes.
//
// One wave per block (four zlib / zstd or five lz4 / snappy waves per CU); a block is processed in windows of
// <= 4 KiB staged in the wave's LDS (one window for the default SstBlockSize):
//   a. matches: every position's longest match among the earlier positions with the same 4-byte hash
//      (hash heads and chains built 64 positions at a time with LDS exchanges; zlib / zstd walk an 8-deep chain of
//      earlier positions, lz4 / snappy take the latest one like lz4_flex / snap), extended 4 bytes a step;
//   b. the parse: one wave-uniform walk over the match bitmap (lane w holds positions [64 w, 64 w + 64):
//      the next match is one ballot away), lazy by one position, the sequences (literal run, length,
//      offset) listed in LDS;
//   c. the codec's elements:
//      lz4 / snappy  lanes size their sequence's elements, a wave scan places them, the wave copies the
//                    literal runs;
//      zlib          one deflate block per window — dynamic Huffman (wave histograms, code lengths by a
//                    bitonic sort + Moffat–Katajainen + a Kraft-sum length limit, the code-length code's
//                    run-length items), fixed Huffman or stored, whichever is shortest; every code's bit
//                    position from prefix sums of code lengths, ORed into the LDS bitstream;
//      zstd          one compressed block per window: Huffman literals (direct weights, 1 or 4 streams
//                    written backwards at suffix-sum bit positions) or raw / RLE literals; sequences with
//                    repeat offsets, each of the LL / OF / ML codes predefined, RLE or FSE_Compressed
//                    (normalised counts + the NCount description) by estimated cost, the three FSE state
//                    machines run side by side on lanes 0-2, their bits placed by a suffix scan;
//                    a raw or RLE block when that is shorter;
//   d. the wave CRC32 of the compressed bytes (chained across windows), the slot written, its length.
//   C2 scan      exclusive scan of the lengths -> out_off (the compressed BlockMeta offsets).
//   C3 pack      one wave per block: slot -> out[out_off[k], out_off[k+1]).
#include <mutex>

#include "sdb_crc.h"
#include "sdb_decode.h"
#include "sdb_device.h"

namespace sdb {

// Phase ticks (diagnostic builds with -DSDB_CZ_PT): s_memtime between marks, summed over waves.
#ifdef SDB_CZ_PT
__device__ unsigned long long g_cz_pt[16];
#define CZ_T0(prev) uint64_t prev = __builtin_amdgcn_s_memtime()
#define CZ_MARK(i, prev)                                                                              \
    do {                                                                                              \
        __builtin_amdgcn_s_waitcnt(0);                                                                \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                             \
        if (lane_id() == 0) atomicAdd(&g_cz_pt[i], (unsigned long long)(t_ - prev));                  \
        prev = t_;                                                                                    \
    } while (0)
#else
#define CZ_T0(prev) \
    do {            \
    } while (0)
#define CZ_MARK(i, prev) \
    do {                 \
    } while (0)
#endif

typedef __attribute__((address_space(3))) uint16_t lu16;
typedef __attribute__((address_space(3))) int16_t li16;
typedef __attribute__((address_space(3))) int32_t li32;

constexpr uint32_t kCzWin = 4096;                   // window: a block of <= 4 KiB is one window
constexpr uint32_t kCzHashBits = 11;
constexpr uint32_t kCzIn = kCzWin + 64;             // the window (+ zeros for reads past its end)
constexpr uint32_t kCzHead = 4u << kCzHashBits;     // u32 hash heads; after the parse: the sequence list
constexpr uint32_t kCzPrev = 2 * kCzWin;            // u16 chain (zlib / zstd); after the parse: entropy scratch
constexpr uint32_t kCzMm = 4 * kCzWin + 128;        // u32 per position; after the parse: out | aux
constexpr uint32_t kCzOutOff = 64;                  // out at mm + 64 (the CRC's 64 zero lead-in bytes before it)
constexpr uint32_t kCzAuxOff = 8192;                // aux at mm + 8 KiB: literal mask, code-length prefix sums, FSE records
constexpr uint32_t kCzOutCap = kCzAuxOff - kCzOutOff;
constexpr uint32_t kCzMaxSeq = kCzHead / 8;         // a match is >= 4 bytes: a window has <= 1024 sequences
constexpr uint32_t kCzMaxMatch = 258;
#ifndef SDB_CZ_NICE
#define SDB_CZ_NICE 128
#endif
#ifndef SDB_CZ_GOOD
#define SDB_CZ_GOOD 16
#endif
constexpr uint32_t kCzNice = SDB_CZ_NICE;           // a chain walk stops at a match this long (zlib level 6)
constexpr uint32_t kCzGood = SDB_CZ_GOOD;           // ... and takes half of its remaining steps past this one

// CRC tables: slicing-by-8 and x^256 only (12 KiB at LDS 0); the six tree-combine steps multiply by their
// constant in registers (gf_mul) instead of reading 24 KiB of tables, which buys a wave per CU (one CRC per
// window, ~600 VALU)
constexpr uint32_t kCzCrcLds = 12 * 1024;

template <uint32_t C>
struct CzCfg {
    static constexpr bool kDeep = C == SDB_CODEC_ZLIB || C == SDB_CODEC_ZSTD;
    static constexpr uint32_t kWaves = kDeep ? 4 : 5;
    // chain depth of zlib / zstd: 8 (r6, scripts/gpu_r6_czdepth.sh, 4 D1 SSTs): zlib 30.4 -> 22.3 ms at ratio
    // 1.0980 -> 1.0971 (zlib level 6: 1.0974), zstd 24.7 -> 15.9 ms at 1.1248 -> 1.1226 (level 3: 1.1309); JSON
    // values zlib 3.73 -> 3.67 (3.75), zstd 3.68 -> 3.63 (3.54).  Depth 4 lost 2-4 % of the ratio on D1.
#ifdef SDB_CZ_DEPTH  // diagnostic knob
    static constexpr uint32_t kDepth = kDeep ? SDB_CZ_DEPTH : 1;
#else
    static constexpr uint32_t kDepth = kDeep ? 8 : 1;
#endif
    static constexpr uint32_t kWaveLds = kCzIn + kCzHead + (kDeep ? kCzPrev : 0) + kCzMm;
    static constexpr uint32_t kLds = kCzCrcLds + kWaves * kWaveLds;
    static_assert(kLds <= 160 * 1024, "compress LDS");
};

// block k's slot in the workspace (rel = block_off[k] - block_off[0]): compressed bytes + CRC stay under
// n + n/8 + 48 for every codec here (literal-only worst cases: lz4 n + n/255 + 10, snappy n + 14, stored
// deflate n + 5 per window + 6, raw zstd n + 3 per window + 12)
__host__ __device__ inline uint64_t cz_slot(uint64_t rel, uint64_t k) { return (rel + rel / 8 + 64 * k + 15) & ~15ull; }

struct CzArgs {
    uint32_t codec;
    const uint8_t *blocks;
    const uint64_t *block_off;  // nblocks + 1
    uint64_t nblocks;
    uint64_t in_bytes;          // block_off[nblocks] - block_off[0] may not exceed it (the slots are sized by it)
    uint8_t *slots;             // workspace
    uint64_t *len;              // nblocks + 1: compressed bytes + CRC per block
    uint8_t *out;
    uint64_t out_cap;
    const uint64_t *out_off;    // nblocks + 1 (the scan)
    unsigned long long *err;
};

SDB_DEV uint32_t lds_u32u(const lu8 *p, uint32_t i) {  // 4 bytes at any LDS byte offset (little-endian)
    const uint32_t a = lds_addr((const void *)(p + i));
    const lu32 *w = (const lu32 *)(uintptr_t)(a & ~3u);
    return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3);
}
SDB_DEV uint64_t lds_u64u(const lu8 *p, uint32_t i) {  // 8 bytes at any LDS byte offset
    const uint32_t a = lds_addr((const void *)(p + i));
    const lu32 *w = (const lu32 *)(uintptr_t)(a & ~3u);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, a & 3) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, a & 3) << 32);
}
SDB_DEV uint32_t cz_hash(uint32_t v) { return (v * 2654435761u) >> (32 - kCzHashBits); }
SDB_DEV uint32_t hibit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }  // v > 0
SDB_DEV uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
SDB_DEV uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

SDB_DEV void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// RFC 1951 3.2.5: length / distance code bases and extra bits
__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
// RFC 8878 3.1.1.3.2.1: literal / match length codes, and the predefined distributions (3.1.1.3.2.2)
__constant__ uint32_t c_zll_base[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                                        20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t c_zll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                       1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t c_zml_base[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,   16,   17,   18,   19,    20,
                                        21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,   34,   35,   37,   39,    41,
                                        43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t c_zml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                       0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t c_zdef[3][53] = {
    {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1},
    {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1},
    {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1}};
// zstd tables in lane order t: 0 literal lengths, 1 match lengths, 2 offsets
__constant__ uint8_t c_zdef_n[3] = {36, 53, 29};
__constant__ uint8_t c_zdef_al[3] = {6, 6, 5};

SDB_DEV uint32_t rev_bits(uint32_t v, uint32_t n) { return __builtin_bitreverse32(v) >> (32 - n); }
// deflate's fixed Huffman code (RFC 1951 3.2.6) of a literal / length symbol: length, and the code
// bit-reversed for the LSB-first stream
SDB_DEV uint32_t fixed_len(uint32_t sym) { return sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8; }
SDB_DEV uint32_t fixed_code(uint32_t sym) {
    if (sym < 144) return rev_bits(0x30 + sym, 8);
    if (sym < 256) return rev_bits(0x190 + sym - 144, 9);
    if (sym < 280) return rev_bits(sym - 256, 7);
    return rev_bits(0xC0 + sym - 280, 8);
}
SDB_DEV uint32_t len_code(uint32_t len) {  // 3..258 -> 0..28
    uint32_t c = 0;
    while (c < 28 && c_len_base[c + 1] <= len) c++;
    return c;
}
SDB_DEV uint32_t dist_code(uint32_t d) {  // 1..32768 -> 0..29
    uint32_t c = 0;
    while (c < 29 && c_dist_base[c + 1] <= d) c++;
    return c;
}
SDB_DEV uint32_t zll_code(uint32_t v) {
    if (v < 16) return v;
    uint32_t c = 16;
    while (c < 35 && c_zll_base[c + 1] <= v) c++;
    return c;
}
SDB_DEV uint32_t zml_code(uint32_t len) {  // match length >= 3
    if (len < 35) return len - 3;
    uint32_t c = 32;
    while (c < 52 && c_zml_base[c + 1] <= len) c++;
    return c;
}

// OR `nb` (<= 32) bits `v` into the LDS bitstream `w` (u32 words, zeroed) at bit position `pos`
SDB_DEV void put_bits(lu32 *w, uint32_t pos, uint32_t v, uint32_t nb) {
    if (!nb) return;
    if (nb < 32) v &= (1u << nb) - 1;
    const uint32_t q = pos >> 5, r = pos & 31;
    __hip_atomic_fetch_or(&w[q], v << r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (r + nb > 32) __hip_atomic_fetch_or(&w[q + 1], v >> (32 - r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

SDB_DEV void cz_crc_tables_to_lds(lu32 *crc) {
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) crc[q] = (&c_crc.t[0][0])[q];
    for (uint32_t q = threadIdx.x; q < 4 * 256; q += blockDim.x) crc[8 * 256 + q] = (&c_mul256.t[0][0])[q];
}
template <int S>
SDB_DEV uint32_t cz_tree_mul(uint32_t c) {
    constexpr uint32_t K = x8n_c(64ull << S);
    return gf_mul(K, c);
}
// crc_tree_combine with the step multipliers in registers
SDB_DEV uint32_t cz_tree_combine(uint32_t c) {
    const uint32_t l = (uint32_t)lane_id();
    uint32_t p = dpp32<0x101>(c);
    if ((l & 1) == 0) c = cz_tree_mul<0>(c) ^ p;
    p = dpp32<0x102>(c);
    if ((l & 3) == 0) c = cz_tree_mul<1>(c) ^ p;
    p = dpp32<0x104>(c);
    if ((l & 7) == 0) c = cz_tree_mul<2>(c) ^ p;
    p = dpp32<0x108>(c);
    if ((l & 15) == 0) c = cz_tree_mul<3>(c) ^ p;
    p = (uint32_t)__builtin_amdgcn_permlane16_swap(c, c, false, false)[1];
    if ((l & 31) == 0) c = cz_tree_mul<4>(c) ^ p;
    p = (uint32_t)__builtin_amdgcn_permlane32_swap(c, c, false, false)[1];
    if (l == 0) c = cz_tree_mul<5>(c) ^ p;
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
}
// wave_crc_image_ra (sdb_crc.h) over the 12 KiB table set
SDB_DEV uint32_t cz_crc_image_ra(const lu8 *img, uint32_t Lc) {
    const uint32_t l = (uint32_t)lane_id();
    const int s = (int)Lc - 64 * (64 - (int)l);
    uint32_t c = 0;
    if (s > -64) {
        const lu128 *w = (const lu128 *)(uintptr_t)(lds_addr((const void *)img) + (uint32_t)(s - (int)(Lc & 15)));
        uint32_t x[20], m[16];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const u32x4 v = w[i];
            x[4 * i] = v.x;
            x[4 * i + 1] = v.y;
            x[4 * i + 2] = v.z;
            x[4 * i + 3] = v.w;
        }
        const uint32_t q = (Lc >> 2) & 3, r = Lc & 3;
        if (q == 0) realign16<0>(x, r, m);
        else if (q == 1) realign16<1>(x, r, m);
        else if (q == 2) realign16<2>(x, r, m);
        else realign16<3>(x, r, m);
        c = crc_seg64_lds(m);
    }
    return cz_tree_combine(c) ^ 0xFFFFFFFFu;
}

// Raw CRC register (init folded in when `first`, no final inversion) of out[0, m) by the wave: out is 16-byte
// aligned with 64 zero bytes before it; bytes past 4096 are copied to `sc` (16-byte aligned, 64 free bytes
// before it).  m <= 4096 + 1024.
SDB_DEV uint32_t cz_crc_raw(lu8 *out, uint32_t m, lu8 *sc, bool first) {
    const uint32_t l = (uint32_t)lane_id();
    if (m < 16) {  // short: lane 0 through the byte table (LDS tables at address 0)
        uint32_t c = 0;
        if (l == 0) {
            const lu32 *t0 = (const lu32 *)(uintptr_t)0;
            c = first ? 0xFFFFFFFFu : 0u;
            for (uint32_t i = 0; i < m; i++) c = (c >> 8) ^ t0[(c ^ out[i]) & 0xFF];
        }
        return uni(c);
    }
    const uint32_t head = m > 4096 ? 4096 : m, tail = m - head;
    if (tail) {
        if (l < 16) ((lu32 *)(sc - 64))[l] = 0;
        for (uint32_t i = l; i < tail; i += 64) sc[i] = out[4096 + i];
    }
    if (first && l == 0) ((lu32 *)out)[0] = ~((const lu32 *)out)[0];  // crc32fast's init, folded into bytes [0, 4)
    wsync();
    uint32_t raw = cz_crc_image_ra(out, head) ^ 0xFFFFFFFFu;
    if (tail) raw = crc_shift_bytes(raw, tail) ^ cz_crc_image_ra(sc, tail) ^ 0xFFFFFFFFu;
    wsync();
    if (first && l == 0) ((lu32 *)out)[0] = ~((const lu32 *)out)[0];
    wsync();
    return raw;
}

// ------------------------------------------------------------------------------------------------
// One lane, any size: a literal-only stream of the codec straight into the global slot (lz4 blocks
// over 4 KiB whose windows find no match to end a sequence).  Returns the bytes written (no CRC).
// ------------------------------------------------------------------------------------------------
SDB_DEV uint32_t cz_literal_only(uint32_t codec, const uint8_t *in, uint32_t n, uint8_t *o) {
    uint32_t p = 0;
    auto lit_copy = [&](const uint8_t *src, uint32_t len) {
        for (uint32_t i = 0; i < len; i++) o[p + i] = src[i];
        p += len;
    };
    if (codec == SDB_CODEC_LZ4) {
        o[0] = (uint8_t)n; o[1] = (uint8_t)(n >> 8); o[2] = (uint8_t)(n >> 16); o[3] = (uint8_t)(n >> 24);
        p = 4;
        o[p++] = (uint8_t)((n >= 15 ? 15 : n) << 4);
        if (n >= 15) {
            uint32_t x = n - 15;
            for (; x >= 255; x -= 255) o[p++] = 255;
            o[p++] = (uint8_t)x;
        }
        lit_copy(in, n);
    }
    return p;
}

// ------------------------------------------------------------------------------------------------
// a. matches over the staged window [0, wn): mm[p] = off << 16 | len (len >= 4 or 0); the returned
//    register is lane w's 64-bit match bitmap of positions [64 w, 64 w + 64).  `room` = bytes from the
//    window start to the block end (lz4's end rules).
// ------------------------------------------------------------------------------------------------
template <uint32_t CODEC>
SDB_DEV uint64_t cz_matches(const lu8 *in, uint32_t wn, uint32_t room, lu32 *head, lu16 *prev, lu32 *mm) {
    constexpr uint32_t kDepth = CzCfg<CODEC>::kDepth;
    const uint32_t l = (uint32_t)lane_id();
    for (uint32_t q = l; q < (1u << kCzHashBits); q += 64) head[q] = 0;
    wsync();
    uint64_t vmask = 0;
    if (wn < 4) return 0;
    const uint32_t last = wn - 4;  // positions with 4 bytes to hash: [0, last]
    // two batches of 64 positions per step: both insert (the second batch after the first, so it sees it),
    // then each lane walks its two chains interleaved (two independent LDS round trips in flight)
    for (uint32_t b0 = 0; b0 <= last; b0 += 128) {
        const uint32_t p0 = b0 + l, p1 = b0 + 64 + l;
        const bool live0 = p0 <= last, live1 = p1 <= last;
        const uint32_t v0 = live0 ? lds_u32u(in, p0) : 0, v1 = live1 ? lds_u32u(in, p1) : 0;
        // the latest earlier position + 1 with this hash: the exchange returns the previous holder, which for
        // lanes of one batch sharing a hash is the lane before (same-address LDS atomics of one instruction
        // are applied in lane order; a candidate not before p is never used, so any other order only loses
        // matches)
        const uint32_t cand0 = live0 ? __hip_atomic_exchange(&head[cz_hash(v0)], p0 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) : 0;
        const uint32_t cand1 = live1 ? __hip_atomic_exchange(&head[cz_hash(v1)], p1 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) : 0;
        if constexpr (kDepth > 1) {
            if (live0) prev[p0] = (uint16_t)cand0;
            if (live1) prev[p1] = (uint16_t)cand1;
        }
        wsync();
        const uint32_t lim0 = live0 ? (wn - p0 < kCzMaxMatch ? wn - p0 : kCzMaxMatch) : 0;
        const uint32_t lim1 = live1 ? (wn - p1 < kCzMaxMatch ? wn - p1 : kCzMaxMatch) : 0;
        uint32_t bl0 = 0, bo0 = 0, c0 = cand0 <= p0 ? cand0 : 0;
        uint32_t bl1 = 0, bo1 = 0, c1 = cand1 <= p1 ? cand1 : 0;
        auto extend = [&](uint32_t q, uint32_t p, uint32_t lim) -> uint32_t {
            uint32_t len = 4;
            while (len < lim) {
                const uint64_t x = lds_u64u(in, q + len) ^ lds_u64u(in, p + len);
                if (x) {
                    len += (uint32_t)__builtin_ctzll(x) >> 3;
                    break;
                }
                len += 8;
            }
            return len < lim ? len : lim;
        };
        // zlib's good / nice lengths: a match of kCzGood bytes cuts the rest of the chain to a half, one of
        // kCzNice ends it
        uint32_t dl0 = kDepth, dl1 = kDepth;
        // inside a run of one byte value (the 4 bytes at p - 1 equal those at p) a match of the run is met at
        // every step of the chain: two steps, as the parse takes such positions only past a match's end
        if (kDepth > 2) {
            if (p0 > 0 && live0 && lds_u32u(in, p0 - 1) == v0) dl0 = 2;
            if (live1 && lds_u32u(in, p1 - 1) == v1) dl1 = 2;
        }
#ifdef SDB_CZ_PT
        uint32_t pt_steps = 0;
#endif
        for (uint32_t d = 0; d < kDepth; d++) {
            if (!c0 && !c1) break;
#ifdef SDB_CZ_PT
            pt_steps++;
#endif
            const uint32_t q0 = c0 ? c0 - 1 : 0, q1 = c1 ? c1 - 1 : 0;
            const uint32_t w0 = lds_u32u(in, q0), w1 = lds_u32u(in, q1);
            uint32_t n0 = 0, n1 = 0;
            if constexpr (kDepth > 1) {
                n0 = prev[q0];
                n1 = prev[q1];
            }
            if (c0 && w0 == v0) {
                const uint32_t len = extend(q0, p0, lim0);
                if (len > bl0) {
                    if (bl0 < kCzGood && len >= kCzGood) dl0 = d + 1 + (kDepth - d - 1) / 2;
                    bl0 = len;
                    bo0 = p0 - q0;
                    if (len >= kCzNice) n0 = 0;
                }
            }
            if (c1 && w1 == v1) {
                const uint32_t len = extend(q1, p1, lim1);
                if (len > bl1) {
                    if (bl1 < kCzGood && len >= kCzGood) dl1 = d + 1 + (kDepth - d - 1) / 2;
                    bl1 = len;
                    bo1 = p1 - q1;
                    if (len >= kCzNice) n1 = 0;
                }
            }
            c0 = c0 && d + 1 < dl0 ? n0 : 0;
            c1 = c1 && d + 1 < dl1 ? n1 : 0;
        }
        auto finish = [&](uint32_t p, bool live, uint32_t blen, uint32_t boff, uint32_t bsel) {
            if (CODEC == SDB_CODEC_LZ4) {  // LZ4: a match starts 12+ bytes before the end, ends 5+ before it
                if (p + 12 > room) blen = 0;
                else if (blen > room - 5 - p) blen = room - 5 - p;
            }
            if (blen < 4) blen = 0;
            if (live) mm[p] = (boff << 16) | blen;
            const uint64_t bits = __ballot(blen >= 4);
            if (l == bsel) vmask = bits;
        };
        finish(p0, live0, bl0, bo0, b0 >> 6);
        finish(p1, live1, bl1, bo1, (b0 >> 6) + 1);
#ifdef SDB_CZ_PT
        {  // 11: wave steps of the chain walks (the slowest lane's), 12: lanes' steps summed
            const uint32_t ws = wave_max(pt_steps);
            const uint32_t ls = wave_sum(pt_steps);
            if (l == 0) {
                atomicAdd(&g_cz_pt[11], (unsigned long long)ws);
                atomicAdd(&g_cz_pt[12], (unsigned long long)ls);
            }
        }
#endif
        wsync();
    }
    return vmask;
}

// b. the greedy parse with one position of lazy evaluation: seq[2 i] = lit | len << 16, seq[2 i + 1] = off
//    (window coordinates).  Returns the sequence count; *tail = the end of the last match.
SDB_DEV uint32_t cz_parse(uint64_t vmask, uint32_t wn, const lu32 *mm, lu32 *seq, uint32_t *tail) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t last = wn >= 4 ? wn - 4 : 0;
    uint32_t nseq = 0, ls = 0, cur = 0;
    while (nseq < kCzMaxSeq && cur < wn && wn >= 4) {
        const uint32_t w0 = cur >> 6;
        const uint64_t mine = l < w0 ? 0 : (l == w0 ? (vmask & (~0ull << (cur & 63))) : vmask);
        const uint64_t any = __ballot(mine != 0);
        if (!any) break;
        const uint32_t ww = (uint32_t)__builtin_ctzll(any);
        const uint64_t mw = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mine >> 32), (int)ww) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, (int)ww);
        const uint32_t q = 64 * ww + (uint32_t)__builtin_ctzll(mw);
        const uint32_t mq = mm[q];
        const uint32_t len = mq & 0xFFFF, off = mq >> 16;
        if (q + 1 <= last && (mm[q + 1] & 0xFFFF) > len) {  // lazy: the next position's match is longer
            cur = q + 1;
            continue;
        }
        if (l == 0) {
            seq[2 * nseq] = (q - ls) | (len << 16);
            seq[2 * nseq + 1] = off;
        }
        nseq++;
        ls = cur = q + len;
    }
    *tail = ls;
    wsync();
    return nseq;
}

// ------------------------------------------------------------------------------------------------
// Huffman code lengths of the symbols with nonzero f[0, ns) (ns <= 512, at least two of them), each
// <= maxlen, by the wave: nonzero (freq << 9 | sym) keys compacted and bitonic-sorted in `work` (>= the
// next power of two of their count); Moffat & Katajainen's method over the sorted run — its first pass on
// lane 0 with the queue heads in registers (Al: >= ns LDS words; the array itself in VGPRs, read by readlane
// at wave-uniform indices, measured four times slower: SGPR spills), its second and third passes as
// wave-parallel pointer jumping and ballot counts — and the Kraft-sum length limit on the per-length
// counts, lengths handed out longest first to the least frequent symbols.  len[0, ns) written (0 for absent symbols).  Returns the max length.
// ------------------------------------------------------------------------------------------------
SDB_DEV uint32_t wave_huff_lengths(const lu32 *f, uint32_t ns, uint32_t maxlen, lu8 *len, lu32 *work, lu32 *Al) {
    const uint32_t l = (uint32_t)lane_id();
    uint32_t m = 0;
    for (uint32_t i0 = 0; i0 < ns; i0 += 64) {
        const uint32_t i = i0 + l;
        const uint32_t fr = i < ns ? f[i] : 0;
        const uint64_t b = __ballot(fr != 0);
        if (fr) work[m + lanes_below(b)] = (fr << 9) | i;
        if (i < ns) len[i] = 0;
        m += (uint32_t)__builtin_popcountll(b);
    }
    uint32_t P = 1;
    while (P < m) P <<= 1;
    for (uint32_t i = m + l; i < P; i += 64) work[i] = 0xFFFFFFFFu;
    wsync();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = l; t < P / 2; t += 64) {
                const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), p = i + j;
                const uint32_t a = work[i], b = work[p];
                if ((a > b) == ((i & k) == 0)) {
                    work[i] = b;
                    work[p] = a;
                }
            }
            wsync();
        }
    }
    if (m == 0) return 0;
    const int n = (int)m;
    if (n == 1) {
        if (l == 0) len[work[0] & 511] = 1;
        wsync();
        return 1;
    }
    // 1. Moffat & Katajainen's first pass on lane 0: the internal nodes' weights, then (once consumed) their
    //    parent indices, in Al[0, n - 1).  The leaves are read from the sorted keys (never written), and the
    //    heads of both queues are kept in registers with the next values loaded ahead, so a pick waits on no
    //    LDS round trip: the head after an internal node is the node behind it (Al, loaded when it became
    //    second) or, when the queue ran dry, the node this step creates.
    if (l == 0) {
        auto LV = [&](int i) -> uint32_t { return i < n ? work[i] >> 9 : 0xFFFFFFFFu; };
        uint32_t l0 = LV(2), l1 = LV(3), l2 = LV(4);
        uint32_t i0 = (work[0] >> 9) + (work[1] >> 9), i1 = 0;
        Al[0] = i0;
        int root = 0, leaf = 2;
        for (int next = 1; next < n - 1; next++) {
            uint32_t w;
            if (leaf >= n || i0 < l0) {
                w = i0;
                Al[root] = (uint32_t)next;
                root++;
                i0 = i1;
                i1 = root + 1 < next ? Al[root + 1] : 0u;
            } else {
                w = l0;
                leaf++;
                l0 = l1;
                l1 = l2;
                l2 = LV(leaf + 2);
            }
            if (leaf >= n || (root < next && i0 < l0)) {
                w += i0;
                Al[root] = (uint32_t)next;
                root++;
                i0 = i1;
                i1 = root + 1 < next ? Al[root + 1] : 0u;
            } else {
                w += l0;
                leaf++;
                l0 = l1;
                l1 = l2;
                l2 = LV(leaf + 2);
            }
            Al[next] = w;
            if (root == next) i0 = w;
            else if (root + 1 == next) i1 = w;
        }
    }
    wsync();
    uint32_t sym[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) sym[k] = 64 * k + l < m ? work[64 * k + l] & 511 : 0;
    wsync();
    // 2. the internal nodes' depths by pointer jumping (the second pass as log2(n) wave-parallel rounds):
    //    D = work, P = Al (the root, node n - 2, is its own parent at depth 0)
    const uint32_t ni = m - 1;
    for (uint32_t i = l; i < ni; i += 64) {
        work[i] = i == ni - 1 ? 0u : 1u;
        if (i == ni - 1) Al[i] = i;
    }
    wsync();
    for (uint32_t r = 1; r < ni; r <<= 1) {
        uint32_t nd[8], np[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t i = 64 * k + l;
            nd[k] = np[k] = 0;
            if (i < ni) {
                const uint32_t pa = Al[i];
                nd[k] = work[i] + work[pa];
                np[k] = Al[pa];
            }
        }
        wsync();
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t i = 64 * k + l;
            if (i < ni) {
                work[i] = nd[k];
                Al[i] = np[k];
            }
        }
        wsync();
    }
    // 3. leaves per depth from the internal nodes' (third pass): with C(d) = internal nodes of depth >= d,
    //    the leaves of depth >= d number 2 C(d - 1) - C(d); the least frequent leaves are the deepest.  Depths
    //    past maxlen are counted at maxlen, then the Kraft-sum fix.
    uint32_t C[17];
    {
        uint32_t dep[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) dep[k] = 64 * k + l < ni ? work[64 * k + l] : 0;
#pragma unroll
        for (uint32_t d = 0; d <= 16; d++) {
            uint32_t c = 0;
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) c += (uint32_t)__builtin_popcountll(__ballot(64 * k + l < ni && dep[k] >= d));
            C[d] = c;
        }
    }
    uint32_t cnt[16], mx = 0;
    {
        auto Lge = [&](uint32_t d) -> uint32_t { return 2 * C[d - 1] - C[d]; };  // 1 <= d <= 16
        cnt[0] = 0;
        for (uint32_t d = 1; d < 16; d++) cnt[d] = 0;
        for (uint32_t d = 1; d < maxlen; d++) cnt[d] = Lge(d) - Lge(d + 1);
        cnt[maxlen] = Lge(maxlen);
        for (uint32_t d = 1; d <= maxlen; d++)
            if (cnt[d]) mx = d;
        if (Lge(maxlen + 1) > 0) {  // deeper leaves: the Kraft-sum limit
            uint32_t total = 0;
            for (uint32_t b = 1; b <= maxlen; b++) total += cnt[b] << (maxlen - b);
            while (total != (1u << maxlen)) {
                cnt[maxlen]--;
                for (uint32_t b = maxlen - 1; b > 0; b--)
                    if (cnt[b]) {
                        cnt[b]--;
                        cnt[b + 1] += 2;
                        break;
                    }
                total--;
            }
            mx = maxlen;
        }
    }
    // leaf j (ascending frequency) -> its length: [0, cnt[maxlen]) maxlen, the next cnt[maxlen - 1] maxlen - 1, ...
    uint32_t end[16];
    {
        uint32_t acc = 0;
        for (int b = 15; b >= 1; b--) {
            if ((uint32_t)b <= maxlen) acc += cnt[b];
            end[b] = acc;
        }
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t j = 64 * k + l;
        if (j < m) {
            uint32_t b = maxlen;
            while (b > 1 && j >= end[b]) b--;
            len[sym[k]] = (uint8_t)b;
        }
    }
    wsync();
    return mx;
}

// deflate's canonical codes (RFC 1951 3.2.2), bit-reversed for the LSB-first stream, by the wave: the
// per-length counts and each symbol's rank among the symbols of its length from ballots.
SDB_DEV void wave_deflate_codes(const lu8 *len, uint32_t ns, lu16 *code) {
    const uint32_t l = (uint32_t)lane_id();
    uint32_t cnt[16];
#pragma unroll
    for (uint32_t b = 0; b < 16; b++) cnt[b] = 0;
    for (uint32_t c0 = 0; c0 < ns; c0 += 64) {
        const uint32_t b = c0 + l < ns ? len[c0 + l] : 0;
#pragma unroll
        for (uint32_t bl = 1; bl < 16; bl++) cnt[bl] += (uint32_t)__builtin_popcountll(__ballot(b == bl));
    }
    uint32_t next[16];
    uint32_t c = 0;
    next[0] = 0;
#pragma unroll
    for (uint32_t b = 1; b < 16; b++) {
        c = (c + (b > 1 ? cnt[b - 1] : 0)) << 1;
        next[b] = c;
    }
    for (uint32_t c0 = 0; c0 < ns; c0 += 64) {
        const uint32_t i = c0 + l;
        const uint32_t b = i < ns ? len[i] : 0;
        uint32_t cv = 0;
#pragma unroll
        for (uint32_t bl = 1; bl < 16; bl++) {
            const uint64_t m = __ballot(b == bl);
            if (b == bl) cv = next[bl] + lanes_below(m);
            next[bl] += (uint32_t)__builtin_popcountll(m);
        }
        if (i < ns) code[i] = b ? (uint16_t)rev_bits(cv, b) : 0;
    }
    wsync();
}

// The mask of literal positions of the window (bit p: not inside a match), the sequence starts from a
// scan.  lmask: 128 words.
SDB_DEV void cz_lit_mask(const lu32 *seq, uint32_t nseq, uint32_t wn, lu32 *lmask) {
    const uint32_t l = (uint32_t)lane_id();
    for (uint32_t q = l; q < 128; q += 64) {
        const uint32_t b0 = 32 * q;
        lmask[q] = b0 + 32 <= wn ? 0xFFFFFFFFu : (b0 >= wn ? 0u : (1u << (wn - b0)) - 1);
    }
    wsync();
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nseq; c0 += 64) {
        const uint32_t i = c0 + l;
        const bool v = i < nseq;
        const uint32_t s0 = v ? seq[2 * i] : 0;
        const uint32_t lit = s0 & 0xFFFF, len = s0 >> 16, span = lit + len;
        const uint32_t inc = wave_incl_scan(span);
        const uint32_t ms = carry + inc - span + lit;  // the match's first position
        for (uint32_t p = ms; p < ms + len;) {
            const uint32_t q = p >> 5, r = p & 31, k = (ms + len - p) < (32 - r) ? (ms + len - p) : (32 - r);
            const uint32_t bits = (k == 32 ? 0xFFFFFFFFu : ((1u << k) - 1)) << r;
            __hip_atomic_fetch_and(&lmask[q], ~bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            p += k;
        }
        carry += wave_readlane(inc, 63);
    }
    wsync();
}

// ------------------------------------------------------------------------------------------------
// zlib: one deflate block for the window, written at bit `origin` of `out` (zeroed past the origin).
// Returns the end bit.  HZ layout (entropy scratch, 8 KiB).
// ------------------------------------------------------------------------------------------------
struct ZlHz {
    lu32 *fq;      // [320]: literal / length 0..285, distances at 288..317
    lu32 *fcl;     // [20]
    lu8 *lens;     // [320]
    lu8 *cll;      // [20]
    lu16 *codes;   // [320]
    lu16 *clc;     // [20]
    lu32 *work;    // [512]
    lu32 *A;       // [320]
    lu16 *rle;     // [320]: sym | extra << 5
    lu32 *misc;    // [32]
    __device__ ZlHz(lu8 *hz)
        : fq((lu32 *)hz), fcl((lu32 *)(hz + 1280)), lens(hz + 1360), cll(hz + 1680), codes((lu16 *)(hz + 1712)),
          clc((lu16 *)(hz + 2352)), work((lu32 *)(hz + 2400)), A((lu32 *)(hz + 4448)), rle((lu16 *)(hz + 5728)),
          misc((lu32 *)(hz + 6368)) {}
};

SDB_DEV uint32_t cz_deflate_window(const lu8 *in, uint32_t wn, const lu32 *seq, uint32_t nseq, lu8 *out,
                                   uint32_t origin, bool final, lu8 *hz_base, lu8 *aux) {
    const uint32_t l = (uint32_t)lane_id();
    ZlHz hz(hz_base);
    lu32 *lmask = (lu32 *)aux;
    lu16 *plen = (lu16 *)aux;
    lu32 *bw = (lu32 *)out;
    CZ_T0(pt);
    for (uint32_t q = l; q < 340; q += 64) hz.fq[q] = 0;  // fq + fcl
    cz_lit_mask(seq, nseq, wn, lmask);
    // histograms: each sequence's length and distance codes, then the literals
    for (uint32_t c0 = 0; c0 < nseq; c0 += 64) {
        const uint32_t i = c0 + l;
        if (i < nseq) {
            const uint32_t s0 = seq[2 * i], off = seq[2 * i + 1];
            __hip_atomic_fetch_add(&hz.fq[257 + len_code(s0 >> 16)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_add(&hz.fq[288 + dist_code(off)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
    }
    for (uint32_t p = l; p < wn; p += 64)
        if ((lmask[p >> 5] >> (p & 31)) & 1)
            __hip_atomic_fetch_add(&hz.fq[in[p]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (l == 0) hz.fq[256] = 1;
    wsync();
    // extra bits (both codes) and the fixed code's size; then >= 2 used symbols per alphabet (the distance
    // alphabet may be unused: two placeholder codes of length 1 keep every code complete)
    uint32_t xb = 0, fixb = 0;
    for (uint32_t s = l; s < 318; s += 64) {
        const uint32_t f = hz.fq[s];
        if (s < 286) fixb += f * fixed_len(s);
        else if (s >= 288) fixb += f * 5;
        if (s >= 257 && s < 286) xb += f * c_len_extra[s - 257];
        if (s >= 288) xb += f * c_dist_extra[s - 288];
    }
    xb = wave_sum(xb);
    fixb = wave_sum(fixb) + xb;
    {
        const uint64_t b = __ballot(l < 30 && hz.fq[288 + l] != 0);
        uint32_t nzl = 0;
        for (uint32_t s = l; s < 286; s += 64) nzl += hz.fq[s] != 0;
        nzl = wave_sum(nzl);
        if (l == 0) {
            uint32_t nz = (uint32_t)__builtin_popcountll(b);
            for (uint32_t t = 0; t < 2 && nz < 2; t++)
                if (!hz.fq[288 + t]) {
                    hz.fq[288 + t] = 1;
                    nz++;
                }
            for (uint32_t t = 0; t < 2 && nzl < 2; t++)  // an empty window: EOB and a placeholder literal
                if (!hz.fq[t]) {
                    hz.fq[t] = 1;
                    nzl++;
                }
        }
        wsync();
    }
    CZ_MARK(5, pt);
    wave_huff_lengths(hz.fq, 286, 15, hz.lens, hz.work, hz.A);
    wave_huff_lengths(hz.fq + 288, 30, 15, hz.lens + 288, hz.work, hz.A);
    CZ_MARK(6, pt);
    // the code-length sequence (HLIT literal / length lengths, then HDIST distance lengths) run-length coded
    uint32_t hlit = 257, hdist = 1;
    for (uint32_t s = l; s < 286; s += 64)
        if (hz.lens[s]) hlit = hlit > s + 1 ? hlit : s + 1;
    if (l < 30 && hz.lens[288 + l]) hdist = l + 1;
    hlit = wave_max(hlit);
    hdist = wave_max(hdist);
    // run-length items (sym | extra << 5) by the wave: run starts from ballots, each start lane sizes and then
    // writes its run's items (16 / 17 / 18 as zlib's send_tree) at a scanned position
    uint32_t nitem = 0;
    {
        const uint32_t N = hlit + hdist;
        auto L = [&](uint32_t i) -> uint32_t { return i < hlit ? hz.lens[i] : hz.lens[288 + i - hlit]; };
        for (uint32_t c0 = 0; c0 < N; c0 += 64) {
            const uint32_t i = c0 + l;
            const bool st = i < N && (i == 0 || L(i) != L(i - 1));
            const uint64_t m = __ballot(st);
            if (l == 0) ((__attribute__((address_space(3))) uint64_t *)(void *)hz.A)[c0 >> 6] = m;  // run-start bitmap
        }
        wsync();
        const __attribute__((address_space(3))) uint64_t *sm = (const __attribute__((address_space(3))) uint64_t *)(void *)hz.A;
        const uint32_t nw = (N + 63) >> 6;
        for (uint32_t c0 = 0; c0 < N; c0 += 64) {
            const uint32_t i = c0 + l;
            const bool st = i < N && ((sm[c0 >> 6] >> l) & 1);
            uint32_t v = 0, run = 0, ni = 0;
            if (st) {
                v = L(i);
                uint32_t w = (i + 1) >> 6, nx = N;
                uint64_t bits = w < nw ? sm[w] & (~0ull << ((i + 1) & 63)) : 0;
                while (!bits && ++w < nw) bits = sm[w];
                if (bits) nx = 64 * w + (uint32_t)__builtin_ctzll(bits);
                run = nx - i;
                uint32_t r = run;
                if (v == 0) {
                    while (r >= 11) { r -= r < 138 ? r : 138; ni++; }
                    if (r >= 3) { ni++; r = 0; }
                    ni += r;
                } else {
                    ni++;
                    r--;
                    while (r >= 3) { r -= r < 6 ? r : 6; ni++; }
                    ni += r;
                }
            }
            const uint32_t inc = wave_incl_scan(ni);
            uint32_t at = nitem + inc - ni;
            if (st) {
                auto emit = [&](uint32_t sym, uint32_t x) {
                    hz.rle[at++] = (uint16_t)(sym | (x << 5));
                    __hip_atomic_fetch_add(&hz.fcl[sym], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                };
                uint32_t r = run;
                if (v == 0) {
                    while (r >= 11) {
                        const uint32_t k = r < 138 ? r : 138;
                        emit(18, k - 11);
                        r -= k;
                    }
                    if (r >= 3) {
                        emit(17, r - 3);
                        r = 0;
                    }
                    for (; r; r--) emit(0, 0);
                } else {
                    emit(v, 0);
                    r--;
                    while (r >= 3) {
                        const uint32_t k = r < 6 ? r : 6;
                        emit(16, k - 3);
                        r -= k;
                    }
                    for (; r; r--) emit(v, 0);
                }
            }
            nitem += wave_readlane(inc, 63);
        }
        wsync();
        if (l == 0) {
            uint32_t nz = 0;
            for (uint32_t s = 0; s < 19; s++) nz += hz.fcl[s] != 0;
            for (uint32_t s = 0; s < 19 && nz < 2; s++)
                if (!hz.fcl[s]) {
                    hz.fcl[s] = 1;
                    nz++;
                }
        }
        wsync();
    }
    CZ_MARK(7, pt);
    wave_huff_lengths(hz.fcl, 19, 7, hz.cll, hz.work, hz.A);
    CZ_MARK(8, pt);
    uint32_t hclen = 19;
    {
        // the dynamic block's size: header + items + codes + extra bits
        uint32_t db = 0;
        for (uint32_t s = l; s < 318; s += 64)
            if (s < 286 || s >= 288) db += hz.fq[s] * hz.lens[s];
        for (uint32_t i = l; i < nitem; i += 64) {
            const uint32_t it = hz.rle[i], sym = it & 31;
            db += hz.cll[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
        }
        db = wave_sum(db);
        const uint64_t nzo = __ballot(l < 19 && hz.cll[c_cl_order[l < 19 ? l : 0]] != 0);
        hclen = nzo ? 64 - (uint32_t)__builtin_clzll(nzo) : 4;
        if (hclen < 4) hclen = 4;
        const uint32_t dynb = 3 + 14 + 3 * hclen + db + xb;
        const uint32_t fb = 3 + fixb;
        const uint32_t sb = ((origin + 3 + 7) & ~7u) - origin + 32 + 8 * wn;
        uint32_t kind = dynb < fb ? 2 : 1;
        if ((kind == 2 ? dynb : fb) >= sb) kind = 0;
        if (kind == 0) {
            // stored: BFINAL / 00, byte-aligned LEN / NLEN and the window's bytes
            if (l == 0) put_bits(bw, origin, final ? 1u : 0u, 3);
            const uint32_t b = (origin + 3 + 7) >> 3;
            wsync();
            if (l == 0) {
                out[b] = (uint8_t)wn; out[b + 1] = (uint8_t)(wn >> 8);
                out[b + 2] = (uint8_t)~wn; out[b + 3] = (uint8_t)(~wn >> 8);
            }
            for (uint32_t i = l; i < wn; i += 64) out[b + 4 + i] = in[i];
            wsync();
            return 8 * (b + 4 + wn);
        }
        if (kind == 1) {
            for (uint32_t s = l; s < 318; s += 64) {
                const bool d = s >= 288;
                hz.lens[s] = (uint8_t)(d ? 5 : (s < 286 ? fixed_len(s) : 0));
                hz.codes[s] = (uint16_t)(d ? rev_bits(s - 288, 5) : (s < 286 ? fixed_code(s) : 0));
            }
            if (l == 0) put_bits(bw, origin, (final ? 1u : 0u) | (1u << 1), 3);
            origin += 3;
        } else {
            wave_deflate_codes(hz.lens, 286, hz.codes);
            wave_deflate_codes(hz.lens + 288, 30, hz.codes + 288);
            wave_deflate_codes(hz.cll, 19, hz.clc);
            if (l == 0) {
                put_bits(bw, origin, (final ? 1u : 0u) | (2u << 1), 3);
                put_bits(bw, origin + 3, (hlit - 257) | ((hdist - 1) << 5) | ((hclen - 4) << 10), 14);
            }
            if (l < hclen) put_bits(bw, origin + 17 + 3 * l, hz.cll[c_cl_order[l]], 3);
            uint32_t pos = origin + 17 + 3 * hclen;
            for (uint32_t c0 = 0; c0 < nitem; c0 += 64) {
                const uint32_t i = c0 + l;
                const uint32_t it = i < nitem ? hz.rle[i] : 0, sym = it & 31, x = it >> 5;
                const uint32_t xn = sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0;
                const uint32_t nb = i < nitem ? hz.cll[sym] + xn : 0;
                const uint32_t inc = wave_incl_scan(nb);
                const uint32_t at = pos + inc - nb;
                if (i < nitem) {
                    put_bits(bw, at, hz.clc[sym], hz.cll[sym]);
                    put_bits(bw, at + hz.cll[sym], x, xn);
                }
                pos += wave_readlane(inc, 63);
            }
            origin = pos;
        }
    }
    wsync();
    CZ_MARK(9, pt);
    // plen[i] = sum of the literal code lengths of bytes [0, i)
    {
        uint32_t carry = 0;
        for (uint32_t c0 = 0; c0 < wn + 1; c0 += 64) {
            const uint32_t i = c0 + l;
            const uint32_t v = i < wn ? hz.lens[in[i]] : 0u;
            const uint32_t inc = wave_incl_scan(v);
            if (i <= wn) plen[i] = (uint16_t)(carry + inc - v);
            carry += wave_readlane(inc, 63);
        }
    }
    wsync();
    uint32_t carry_bits = origin, carry_pos = 0;
    for (uint32_t c0 = 0; c0 < nseq; c0 += 64) {
        const uint32_t i = c0 + l;
        const bool v = i < nseq;
        const uint32_t s0 = v ? seq[2 * i] : 0, off = v ? seq[2 * i + 1] : 0;
        const uint32_t lit = s0 & 0xFFFF, len = s0 >> 16, span = lit + len;
        const uint32_t pinc = wave_incl_scan(span);
        const uint32_t lstart = carry_pos + pinc - span;
        uint32_t lbits = 0, dbits = 0, lval = 0, dval = 0;
        if (v) {
            const uint32_t lc = len_code(len), dc = dist_code(off);
            lval = hz.codes[257 + lc] | ((len - c_len_base[lc]) << hz.lens[257 + lc]);
            lbits = hz.lens[257 + lc] + c_len_extra[lc];
            dval = hz.codes[288 + dc] | ((off - c_dist_base[dc]) << hz.lens[288 + dc]);
            dbits = hz.lens[288 + dc] + c_dist_extra[dc];
        }
        const uint32_t litb = v ? (uint32_t)(plen[lstart + lit] - plen[lstart]) : 0;
        const uint32_t bits = litb + lbits + dbits;
        const uint32_t binc = wave_incl_scan(bits);
        const uint32_t bstart = carry_bits + binc - bits;
        if (v) {
            put_bits(bw, bstart + litb, lval, lbits);
            put_bits(bw, bstart + litb + lbits, dval, dbits);
        }
        const uint32_t ncur = nseq - c0 < 64 ? nseq - c0 : 64;
        for (uint32_t j = 0; j < ncur; j++) {
            const uint32_t ls_j = (uint32_t)__builtin_amdgcn_readlane((int)lstart, (int)j);
            const uint32_t lit_j = (uint32_t)__builtin_amdgcn_readlane((int)lit, (int)j);
            const uint32_t b_j = (uint32_t)__builtin_amdgcn_readlane((int)bstart, (int)j);
            for (uint32_t x = l; x < lit_j; x += 64) {
                const uint32_t c = in[ls_j + x];
                put_bits(bw, b_j + (plen[ls_j + x] - plen[ls_j]), hz.codes[c], hz.lens[c]);
            }
        }
        carry_bits += wave_readlane(binc, 63);
        carry_pos += wave_readlane(pinc, 63);
    }
    // final literals [carry_pos, wn), then end-of-block
    for (uint32_t x = l; x < wn - carry_pos; x += 64) {
        const uint32_t c = in[carry_pos + x];
        put_bits(bw, carry_bits + (plen[carry_pos + x] - plen[carry_pos]), hz.codes[c], hz.lens[c]);
    }
    carry_bits += plen[wn] - plen[carry_pos];
    if (l == 0) put_bits(bw, carry_bits, hz.codes[256], hz.lens[256]);
    carry_bits += hz.lens[256];
    wsync();
    CZ_MARK(10, pt);
    return carry_bits;
}

// ------------------------------------------------------------------------------------------------
// zstd: one block for the window, its content written at out[ob, ...) (zeroed).  Returns the content size
// (0: not smaller than the window — the caller writes a raw block).  rep: the repeat offsets, carried.
// HZ layout (8 KiB): lit [0, 4096) then the FSE tables; fq / code histograms + norms [4096, 5120);
// Huffman lens [5120, 5376), codes [5376, 5888); work [5888, 7936); misc [7936, 8192).
// ------------------------------------------------------------------------------------------------
SDB_DEV void fse_build_ct(const li16 *norm, uint32_t ns, uint32_t al, lu16 *stab, li32 *tt, lu8 *spread, lu16 *cumul) {
    const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t high = size - 1;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= ns; u++) {
        const int nc = norm[u - 1];
        if (nc == -1) {
            cumul[u] = cumul[u - 1] + 1;
            spread[high--] = (uint8_t)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (uint32_t)nc;
        }
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s < ns; s++) {
        const int nc = norm[s];
        for (int i = 0; i < nc; i++) {
            spread[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    }
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t s = spread[u];
        stab[cumul[s]] = (uint16_t)(size + u);
        cumul[s] = cumul[s] + 1;
    }
    int total = 0;
    for (uint32_t s = 0; s < ns; s++) {
        const int nc = norm[s];
        if (nc == 0) {
            tt[2 * s] = (int32_t)(((al + 1) << 16) - size);
            tt[2 * s + 1] = 0;
        } else if (nc == -1 || nc == 1) {
            tt[2 * s] = (int32_t)((al << 16) - size);
            tt[2 * s + 1] = total - 1;
            total++;
        } else {
            const uint32_t mbo = al - hibit((uint32_t)nc - 1), msp = (uint32_t)nc << mbo;
            tt[2 * s] = (int32_t)((mbo << 16) - msp);
            tt[2 * s + 1] = total - nc;
            total += nc;
        }
    }
}

// FSE table description (RFC 8878 4.1.1) of norm[0, ns) at accuracy log al into o; returns its bytes.
SDB_DEV uint32_t fse_ncount(const li16 *norm, uint32_t ns, uint32_t al, lu8 *o) {
    uint64_t bs = al - 5;
    uint32_t bc = 4, op = 0;
    int remaining = (1 << al) + 1, threshold = 1 << al, nb = (int)al + 1;
    uint32_t sym = 0;
    bool prev0 = false;
    auto flush = [&]() {
        while (bc >= 8) {
            o[op++] = (uint8_t)bs;
            bs >>= 8;
            bc -= 8;
        }
    };
    while (sym < ns && remaining > 1) {
        if (prev0) {
            uint32_t start = sym;
            while (sym < ns && !norm[sym]) sym++;
            while (sym >= start + 24) {
                start += 24;
                bs |= 0xFFFFull << bc;
                bc += 16;
                flush();
            }
            while (sym >= start + 3) {
                start += 3;
                bs |= 3ull << bc;
                bc += 2;
            }
            bs |= (uint64_t)(sym - start) << bc;
            bc += 2;
            flush();
        }
        int count = norm[sym++];
        const int mx = 2 * threshold - 1 - remaining;
        remaining -= count < 0 ? -count : count;
        count++;
        if (count >= threshold) count += mx;
        bs |= (uint64_t)(uint32_t)count << bc;
        bc += (uint32_t)nb;
        bc -= count < mx ? 1u : 0u;
        prev0 = count == 1;
        while (remaining < threshold) {
            nb--;
            threshold >>= 1;
        }
        flush();
    }
    if (bc) o[op++] = (uint8_t)bs;
    return op;
}

// A serial forward bitstream (one lane) into LDS bytes: BIT_addBits / BIT_closeCStream.
struct SerBits {
    lu8 *o;
    uint32_t op = 0, bc = 0;
    uint64_t acc = 0;
    __device__ explicit SerBits(lu8 *out) : o(out) {}
    __device__ void add(uint32_t v, uint32_t nb) {
        if (nb < 32) v &= (1u << nb) - 1;
        acc |= (uint64_t)v << bc;
        bc += nb;
        while (bc >= 8) {
            o[op++] = (uint8_t)acc;
            acc >>= 8;
            bc -= 8;
        }
    }
    __device__ uint32_t close() {  // the end mark, then the partial byte
        add(1u, 1);
        if (bc) o[op++] = (uint8_t)acc;
        return op;
    }
};

// Huffman weights wt[0, N) (N >= 2, values 0..11) as an FSE-compressed tree description (RFC 8878 4.2.1.2:
// NCount at accuracy log <= 6, then two interleaved states sharing the table — HUF_compressWeights /
// FSE_compress_usingCTable): bytes into o, or 0 when the weights do not compress that way (one value, every
// value once, or >= 128 bytes).  One lane; scratch: 640 bytes.
SDB_DEV uint32_t huf_weights_fse(const lu8 *wt, uint32_t N, lu8 *o, lu8 *scratch) {
    li16 *norm = (li16 *)scratch;                 // [16]
    lu16 *stab = (lu16 *)(scratch + 32);          // [64]
    li32 *tt = (li32 *)(scratch + 160);           // [16][2]
    lu8 *spread = scratch + 288;                  // [64]
    lu16 *cumul = (lu16 *)(scratch + 352);        // [17]
    uint32_t cnt[12];
    for (uint32_t w = 0; w < 12; w++) cnt[w] = 0;
    for (uint32_t i = 0; i < N; i++) cnt[wt[i]]++;
    uint32_t maxw = 0, maxc = 0, best = 0;
    for (uint32_t w = 0; w < 12; w++)
        if (cnt[w]) {
            maxw = w;
            if (cnt[w] > maxc) {
                maxc = cnt[w];
                best = w;
            }
        }
    if (maxc == N || maxc == 1) return 0;
    uint32_t al = hibit(N - 1);
    al = al > 2 ? al - 2 : 0;
    if (al > 6) al = 6;
    const uint32_t a1 = hibit(N) + 1, a2 = hibit(maxw ? maxw : 1) + 2, minb = a1 < a2 ? a1 : a2;
    if (al < minb) al = minb;
    if (al < 5) al = 5;
    if (al > 6) al = 6;
    const int scale = 1 << al;
    int sum = 0;
    for (uint32_t w = 0; w <= maxw; w++) {
        int v = 0;
        if (cnt[w]) {
            v = (int)(((uint32_t)cnt[w] * (uint32_t)scale + N / 2) / N);
            if (v < 1) v = 1;
        }
        norm[w] = (int16_t)v;
        sum += v;
    }
    int diff = scale - sum;
    if (diff >= 0 || norm[best] + diff >= 1) {
        norm[best] = (int16_t)(norm[best] + diff);
    } else {
        while (diff < 0) {
            uint32_t m = 0;
            for (uint32_t w = 0; w <= maxw; w++)
                if (norm[w] > norm[m]) m = w;
            norm[m] = (int16_t)(norm[m] - 1);
            diff++;
        }
    }
    const uint32_t hs = fse_ncount(norm, maxw + 1, al, o);
    fse_build_ct(norm, maxw + 1, al, stab, tt, spread, cumul);
    SerBits bs(o + hs);
    uint32_t st[2];  // st[0]: even indices (state 1), st[1]: odd (state 2)
    auto init = [&](uint32_t sym) -> uint32_t {
        const int dnb = tt[2 * sym], dfs = tt[2 * sym + 1];
        const uint32_t nbo = (uint32_t)((dnb + (1 << 15)) >> 16);
        const uint32_t v = (nbo << 16) - (uint32_t)dnb;
        return stab[(int)(v >> nbo) + dfs];
    };
    st[(N - 1) & 1] = init(wt[N - 1]);
    st[(N - 2) & 1] = init(wt[N - 2]);
    for (int i = (int)N - 3; i >= 0; i--) {
        const uint32_t sym = wt[i], k = (uint32_t)i & 1;
        const int dnb = tt[2 * sym], dfs = tt[2 * sym + 1];
        const uint32_t nb = (uint32_t)((int)st[k] + dnb) >> 16;
        bs.add(st[k], nb);
        st[k] = stab[(int)(st[k] >> nb) + dfs];
        if (hs + bs.op > 120) return 0;
    }
    bs.add(st[1] - (uint32_t)scale, al);
    bs.add(st[0] - (uint32_t)scale, al);
    const uint32_t total = hs + bs.close();
    return total < 128 ? total : 0;
}

struct ZsHz {
    lu8 *lit;      // [4096]
    lu16 *stab;    // [3][256] (over lit, after the literals section)
    li32 *tt;      // [3][64][2]
    lu8 *spread;   // [3][256]
    lu8 *nc;       // [3][64]: NCount descriptions
    lu32 *fq;      // [256] literal histogram; then [3][64] code histograms
    li16 *norm;    // [3][64] (at fq + 768 B)
    lu8 *lens;     // [256]
    lu16 *codes;   // [256]
    lu32 *work;    // [512]: sort + MK; then cumul [3][66] u16
    lu32 *misc;    // [64]: scalars, then (byte 64 on) the FSE tree description
    __device__ ZsHz(lu8 *hz)
        : lit(hz), stab((lu16 *)hz), tt((li32 *)(hz + 1536)), spread(hz + 3072), nc(hz + 3840), fq((lu32 *)(hz + 4096)),
          norm((li16 *)(hz + 4096 + 768)), lens(hz + 5120), codes((lu16 *)(hz + 5376)), work((lu32 *)(hz + 5888)),
          misc((lu32 *)(hz + 7936)) {}
};

// The per-table work of lane t (0 LL, 1 ML, 2 OF): the mode by estimated cost, the table description,
// the encoding table.  Returns mode | al << 8 | ncount bytes << 16.
SDB_DEV uint32_t zs_table(ZsHz &hz, uint32_t t, uint32_t nseq) {
    lu32 *f = hz.fq + 64 * t;
    li16 *norm = hz.norm + 64 * t;
    const uint32_t ns_max = c_zdef_n[t];
    uint32_t maxsym = 0, nz = 0, best = 0;
    for (uint32_t s = 0; s < ns_max; s++)
        if (f[s]) {
            maxsym = s;
            nz++;
            if (f[s] > f[best] || !f[best]) best = s;
        }
    lu16 *cumul = (lu16 *)hz.work + 66 * t;
    if (nz == 1) {  // RLE: the one code as the description, no state bits
        hz.nc[64 * t] = (uint8_t)maxsym;
        return 1u | (0u << 8) | (1u << 16);
    }
    // predefined cost (bits, fixed point 1/256)
    const uint32_t dal = c_zdef_al[t];
    float pre = 0.f;
    for (uint32_t s = 0; s <= maxsym; s++)
        if (f[s]) {
            const int d = c_zdef[t][s];
            pre += (float)f[s] * ((float)dal - __log2f((float)(d < 0 ? 1 : d)));
        }
    // custom: the accuracy log as zstd's FSE_optimalTableLog, counts normalised to 2^al, every used code >= 1
    const uint32_t maxal = t == 2 ? 8 : 9;
    uint32_t al = nseq > 1 ? hibit(nseq - 1) : 0;
    al = al > 2 ? al - 2 : 0;
    if (al > maxal) al = maxal;
    const uint32_t a1 = hibit(nseq) + 1, a2 = hibit(maxsym ? maxsym : 1) + 2, minb = a1 < a2 ? a1 : a2;
    if (al < minb) al = minb;
    if (al < 5) al = 5;
    if (al > 8) al = 8;
    const int scale = 1 << al;
    int sum = 0;
    for (uint32_t s = 0; s <= maxsym; s++) {
        int v = 0;
        if (f[s]) {
            v = (int)(((uint64_t)f[s] * (uint32_t)scale + nseq / 2) / nseq);
            if (v < 1) v = 1;
        }
        norm[s] = (int16_t)v;
        sum += v;
    }
    int diff = scale - sum;
    if (diff >= 0 || norm[best] + diff >= 1) {
        norm[best] = (int16_t)(norm[best] + diff);
    } else {
        while (diff < 0) {
            uint32_t m = 0;
            for (uint32_t s = 0; s <= maxsym; s++)
                if (norm[s] > norm[m]) m = s;
            norm[m] = (int16_t)(norm[m] - 1);
            diff++;
        }
    }
    float cus = 0.f;
    for (uint32_t s = 0; s <= maxsym; s++)
        if (f[s]) cus += (float)f[s] * ((float)al - __log2f((float)norm[s]));
    const uint32_t ncb = fse_ncount(norm, maxsym + 1, al, hz.nc + 64 * t);
    cus += 8.f * (float)ncb;
    if (pre <= cus) {
        for (uint32_t s = 0; s < ns_max; s++) norm[s] = c_zdef[t][s];
        fse_build_ct(norm, ns_max, dal, hz.stab + 256 * t, hz.tt + 128 * t, hz.spread + 256 * t, cumul);
        return 0u | (dal << 8);
    }
    fse_build_ct(norm, maxsym + 1, al, hz.stab + 256 * t, hz.tt + 128 * t, hz.spread + 256 * t, cumul);
    return 2u | (al << 8) | (ncb << 16);
}

SDB_DEV uint32_t cz_zstd_window(const lu8 *in, uint32_t wn, lu32 *seq, uint32_t nseq, lu8 *out, uint32_t ob,
                                uint32_t (&rep)[3], lu8 *hz_base, lu8 *aux) {
    const uint32_t l = (uint32_t)lane_id();
    ZsHz hz(hz_base);
    lu32 *lmask = (lu32 *)aux;
    lu16 *plen = (lu16 *)aux;
    lu16 *fsei = (lu16 *)aux;  // [3][1024]
    lu32 *bw = (lu32 *)out;
    for (uint32_t q = l; q < 256; q += 64) hz.fq[q] = 0;
    cz_lit_mask(seq, nseq, wn, lmask);
    // literals gathered in order, their histogram
    uint32_t nlit = 0;
    for (uint32_t c0 = 0; c0 < wn; c0 += 64) {
        const uint32_t p = c0 + l;
        const bool isl = p < wn && ((lmask[p >> 5] >> (p & 31)) & 1);
        const uint64_t b = __ballot(isl);
        if (isl) {
            const uint32_t c = in[p];
            hz.lit[nlit + lanes_below(b)] = (uint8_t)c;
            __hip_atomic_fetch_add(&hz.fq[c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        nlit += (uint32_t)__builtin_popcountll(b);
    }
    wsync();
    // ---- literals section
    uint32_t nz = 0, maxsym = 0;
    for (uint32_t s = l; s < 256; s += 64)
        if (hz.fq[s]) {
            nz++;
            maxsym = s;
        }
    nz = wave_sum(nz);
    maxsym = wave_max(maxsym);
    const uint32_t raw_hdr = nlit < 32 ? 1 : (nlit < 4096 ? 2 : 3);
    uint32_t p = ob;  // output byte position
    bool huf = false;
    uint32_t maxbits = 0;
    uint32_t td = 0;  // the tree description's bytes: direct weights, or FSE-compressed (hz.misc byte 16 on)
    bool tfse = false;
    // the literals' order-0 entropy (bits, x16) bounds what a Huffman code can save: skip the code when even
    // the entropy plus a tree description would not beat raw literals (random bytes, D1's values)
    uint32_t hfx = 0;
    for (uint32_t s = l; s < 256; s += 64) {
        const uint32_t f = hz.fq[s];
        if (f) hfx += (uint32_t)(16.f * (float)f * __log2f((float)nlit / (float)f));
    }
    hfx = wave_sum(hfx);
    if (nz >= 2 && nlit >= 64 && hfx / 128 + 40 < nlit) {
        maxbits = wave_huff_lengths(hz.fq, maxsym + 1, 11, hz.lens, hz.work, hz.work + 256);
        uint32_t bits = 0;
        for (uint32_t s = l; s <= maxsym; s += 64) bits += hz.fq[s] * hz.lens[s];
        bits = wave_sum(bits);
        // weights of symbols 0 .. maxsym - 1 (the last one's is implied) into work, then the FSE description
        lu8 *wt = (lu8 *)hz.work;
        for (uint32_t s = l; s < maxsym; s += 64) wt[s] = hz.lens[s] ? (uint8_t)(maxbits + 1 - hz.lens[s]) : 0;
        wsync();
        if (l == 0) {
            const uint32_t f = huf_weights_fse(wt, maxsym, (lu8 *)hz.misc + 64, (lu8 *)hz.work + 256);
            const uint32_t direct = maxsym <= 128 ? 1 + (maxsym + 1) / 2 : 0;
            uint32_t r = 0;
            if (f && (!direct || f + 1 < direct)) r = (f + 1) | (1u << 16);
            else if (direct) r = direct;
            hz.misc[0] = r;
        }
        wsync();
        td = hz.misc[0] & 0xFFFF;
        tfse = (hz.misc[0] >> 16) != 0;
        const uint32_t est = 3 + td + (nlit < 256 ? 0 : 6 + 4) + bits / 8 + 1;
        huf = td && est + 8 < raw_hdr + nlit;
    }
    if (nlit == 0 || nz == 1) {
        const uint32_t type = nz == 1 ? 1u : 0u;
        if (l == 0) {
            if (raw_hdr == 1) out[p] = (uint8_t)(type | (nlit << 3));
            else if (raw_hdr == 2) {
                const uint32_t h = type | (1u << 2) | (nlit << 4);
                out[p] = (uint8_t)h; out[p + 1] = (uint8_t)(h >> 8);
            } else {
                const uint32_t h = type | (3u << 2) | (nlit << 4);
                out[p] = (uint8_t)h; out[p + 1] = (uint8_t)(h >> 8); out[p + 2] = (uint8_t)(h >> 16);
            }
            if (nz == 1) out[p + raw_hdr] = hz.lit[0];
        }
        p += raw_hdr + (nz == 1 ? 1 : 0);
    } else if (!huf) {
        if (l == 0) {
            if (raw_hdr == 1) out[p] = (uint8_t)(nlit << 3);
            else if (raw_hdr == 2) {
                const uint32_t h = (1u << 2) | (nlit << 4);
                out[p] = (uint8_t)h; out[p + 1] = (uint8_t)(h >> 8);
            } else {
                const uint32_t h = (3u << 2) | (nlit << 4);
                out[p] = (uint8_t)h; out[p + 1] = (uint8_t)(h >> 8); out[p + 2] = (uint8_t)(h >> 16);
            }
        }
        for (uint32_t i = l; i < nlit; i += 64) out[p + raw_hdr + i] = hz.lit[i];
        p += raw_hdr + nlit;
    } else {
        // zstd's canonical codes: weight w = maxbits + 1 - len; within the index space, weight-1 symbols
        // first (in symbol order), then weight 2, ...; code = start >> (w - 1) (HUF_readDTableX1)
        if (l == 0) {
            uint32_t cnt[13], start[13];
            for (uint32_t w = 0; w < 13; w++) cnt[w] = 0;
            for (uint32_t s = 0; s <= maxsym; s++)
                if (hz.lens[s]) cnt[maxbits + 1 - hz.lens[s]]++;
            uint32_t acc = 0;
            for (uint32_t w = 1; w <= maxbits; w++) {
                start[w] = acc;
                acc += cnt[w] << (w - 1);
            }
            for (uint32_t s = 0; s <= maxsym; s++) {
                const uint32_t b = hz.lens[s];
                if (!b) {
                    hz.codes[s] = 0;
                    continue;
                }
                const uint32_t w = maxbits + 1 - b;
                hz.codes[s] = (uint16_t)(start[w] >> (w - 1));
                start[w] += 1u << (w - 1);
            }
        }
        wsync();
        // plen over the literals
        {
            uint32_t carry = 0;
            for (uint32_t c0 = 0; c0 < nlit + 1; c0 += 64) {
                const uint32_t i = c0 + l;
                const uint32_t v = i < nlit ? hz.lens[hz.lit[i]] : 0u;
                const uint32_t inc = wave_incl_scan(v);
                if (i <= nlit) plen[i] = (uint16_t)(carry + inc - v);
                carry += wave_readlane(inc, 63);
            }
        }
        wsync();
        const uint32_t ns = nlit < 256 ? 1 : 4, seg = ns == 1 ? nlit : (nlit + 3) / 4;
        uint32_t sbytes[4] = {0, 0, 0, 0}, sa[4], sb[4], comp = td + (ns == 4 ? 6 : 0);
        for (uint32_t k = 0; k < ns; k++) {
            sa[k] = k * seg;
            sb[k] = k + 1 == ns ? nlit : (k + 1) * seg;
            sbytes[k] = (plen[sb[k]] - plen[sa[k]]) / 8 + 1;
            comp += sbytes[k];
        }
        const uint32_t sf = ns == 1 ? 0 : (nlit <= 1023 && comp <= 1023 ? 1 : 2);
        const uint32_t lh = sf == 2 ? 4 : 3;
        if (l == 0) {
            if (sf == 2) {
                const uint32_t h = 2u | (2u << 2) | (nlit << 4) | (comp << 18);
                out[p] = (uint8_t)h; out[p + 1] = (uint8_t)(h >> 8); out[p + 2] = (uint8_t)(h >> 16); out[p + 3] = (uint8_t)(h >> 24);
            } else {
                const uint32_t h = 2u | (sf << 2) | (nlit << 4) | (comp << 14);
                out[p] = (uint8_t)h; out[p + 1] = (uint8_t)(h >> 8); out[p + 2] = (uint8_t)(h >> 16);
            }
            out[p + lh] = (uint8_t)(tfse ? td - 1 : 127 + maxsym);
        }
        if (tfse) {  // FSE-compressed weights: the header byte is their size
            for (uint32_t i = l; i + 1 < td; i += 64) out[p + lh + 1 + i] = ((lu8 *)hz.misc)[64 + i];
        } else {
            // direct weights: symbols 0 .. maxsym - 1, two per byte (the first in the high nibble)
            for (uint32_t i = l; i < (maxsym + 1) / 2; i += 64) {
                const uint32_t s0 = 2 * i, s1 = 2 * i + 1;
                const uint32_t w0 = hz.lens[s0] ? maxbits + 1 - hz.lens[s0] : 0;
                const uint32_t w1 = s1 < maxsym && hz.lens[s1] ? maxbits + 1 - hz.lens[s1] : 0;
                out[p + lh + 1 + i] = (uint8_t)((w0 << 4) | w1);
            }
        }
        uint32_t s0 = p + lh + td;
        if (ns == 4 && l == 0) {
            out[s0] = (uint8_t)sbytes[0]; out[s0 + 1] = (uint8_t)(sbytes[0] >> 8);
            out[s0 + 2] = (uint8_t)sbytes[1]; out[s0 + 3] = (uint8_t)(sbytes[1] >> 8);
            out[s0 + 4] = (uint8_t)sbytes[2]; out[s0 + 5] = (uint8_t)(sbytes[2] >> 8);
        }
        if (ns == 4) s0 += 6;
        wsync();
        uint32_t sbase[4];
        sbase[0] = s0;
        for (uint32_t k = 1; k < ns; k++) sbase[k] = sbase[k - 1] + sbytes[k - 1];
        // symbol j of stream k at bit plen[b_k] - plen[j + 1] (written last to first), the end mark after
        for (uint32_t j = l; j < nlit; j += 64) {
            const uint32_t k = ns == 1 ? 0 : (j / seg < 3 ? j / seg : 3);
            const uint32_t kb = k == 0 ? sb[0] : k == 1 ? sb[1] : k == 2 ? sb[2] : sb[3];
            const uint32_t kbase = k == 0 ? sbase[0] : k == 1 ? sbase[1] : k == 2 ? sbase[2] : sbase[3];
            const uint32_t c = hz.lit[j];
            put_bits(bw, 8 * kbase + (plen[kb] - plen[j + 1]), hz.codes[c], hz.lens[c]);
        }
        if (l < ns) {
            const uint32_t kb = l == 0 ? sb[0] : l == 1 ? sb[1] : l == 2 ? sb[2] : sb[3];
            const uint32_t ka = l == 0 ? sa[0] : l == 1 ? sa[1] : l == 2 ? sa[2] : sa[3];
            const uint32_t kbase = l == 0 ? sbase[0] : l == 1 ? sbase[1] : l == 2 ? sbase[2] : sbase[3];
            put_bits(bw, 8 * kbase + (plen[kb] - plen[ka]), 1u, 1);
        }
        wsync();
        p = s0 + comp - (td + (ns == 4 ? 6 : 0));
    }
    // ---- sequences section
    if (l == 0) {
        if (nseq < 128) out[p] = (uint8_t)nseq;
        else {
            out[p] = (uint8_t)((nseq >> 8) + 128);
            out[p + 1] = (uint8_t)nseq;
        }
    }
    p += nseq < 128 ? 1 : 2;
    if (nseq) {
        // repeat offsets (RFC 8878 3.1.2.5), serial: seq[2 i + 1] = offBase | llc << 16 | mlc << 22
        if (l == 0) {
            uint32_t r0 = rep[0], r1 = rep[1], r2 = rep[2];
            for (uint32_t i = 0; i < nseq; i++) {
                const uint32_t s0 = seq[2 * i], lit = s0 & 0xFFFF, off = seq[2 * i + 1];
                uint32_t obase;
                if (lit) obase = off == r0 ? 1 : off == r1 ? 2 : off == r2 ? 3 : off + 3;
                else obase = off == r1 ? 1 : off == r2 ? 2 : off == r0 - 1 ? 3 : off + 3;
                if (obase > 3) {
                    r2 = r1;
                    r1 = r0;
                    r0 = off;
                } else {
                    const uint32_t idx = lit ? obase - 1 : obase;
                    if (idx == 1) {
                        r1 = r0;
                        r0 = off;
                    } else if (idx == 2) {
                        r2 = r1;
                        r1 = r0;
                        r0 = off;
                    } else if (idx == 3) {
                        r2 = r1;
                        r1 = r0;
                        r0 = off;
                    }
                }
                seq[2 * i + 1] = obase;
            }
            hz.misc[0] = r0;
            hz.misc[1] = r1;
            hz.misc[2] = r2;
        }
        for (uint32_t q = l; q < 3 * 64; q += 64) hz.fq[q] = 0;
        wsync();
        rep[0] = hz.misc[0];
        rep[1] = hz.misc[1];
        rep[2] = hz.misc[2];
        for (uint32_t i = l; i < nseq; i += 64) {
            const uint32_t s0 = seq[2 * i], obase = seq[2 * i + 1];
            const uint32_t llc = zll_code(s0 & 0xFFFF), mlc = zml_code(s0 >> 16), ofc = hibit(obase);
            seq[2 * i + 1] = obase | (llc << 16) | (mlc << 22);
            __hip_atomic_fetch_add(&hz.fq[llc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_add(&hz.fq[64 + mlc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_add(&hz.fq[128 + ofc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        wsync();
        // the three tables side by side on lanes 0-2, then their state machines (last sequence first)
        if (l < 3) {
            const uint32_t r = zs_table(hz, l, nseq);
            hz.misc[4 + l] = r;
            const uint32_t mode = r & 0xFF, al = (r >> 8) & 0xFF;
            uint32_t fin = 0;
            if (mode != 1) {
                const lu16 *stab = hz.stab + 256 * l;
                const li32 *tt = hz.tt + 128 * l;
                auto code_of = [&](uint32_t n) -> uint32_t {
                    const uint32_t w = seq[2 * n + 1];
                    return l == 0 ? (w >> 16) & 63 : l == 1 ? (w >> 22) & 63 : hibit(w & 0xFFFF);
                };
                uint32_t c = code_of(nseq - 1);
                int dnb = tt[2 * c], dfs = tt[2 * c + 1];
                const uint32_t nbo = (uint32_t)((dnb + (1 << 15)) >> 16);
                uint32_t value = (nbo << 16) - (uint32_t)dnb;
                value = stab[(int)(value >> nbo) + dfs];
                for (int n = (int)nseq - 2; n >= 0; n--) {
                    c = code_of((uint32_t)n);
                    dnb = tt[2 * c];
                    dfs = tt[2 * c + 1];
                    const uint32_t nb = (uint32_t)((int)value + dnb) >> 16;
                    fsei[1024 * l + n] = (uint16_t)((nb << 12) | (value & ((1u << nb) - 1)));
                    value = stab[(int)(value >> nb) + dfs];
                }
                fin = value - (1u << al);
            } else {
                for (uint32_t n = 0; n + 1 < nseq; n++) fsei[1024 * l + n] = 0;
            }
            hz.misc[8 + l] = fin;
        }
        wsync();
        const uint32_t r_ll = hz.misc[4], r_ml = hz.misc[5], r_of = hz.misc[6];
        const uint32_t m_ll = r_ll & 0xFF, m_ml = r_ml & 0xFF, m_of = r_of & 0xFF;
        const uint32_t al_ll = m_ll == 1 ? 0 : (r_ll >> 8) & 0xFF, al_ml = m_ml == 1 ? 0 : (r_ml >> 8) & 0xFF,
                       al_of = m_of == 1 ? 0 : (r_of >> 8) & 0xFF;
        const uint32_t n_ll = r_ll >> 16, n_ml = r_ml >> 16, n_of = r_of >> 16;
        // modes byte, then the descriptions in the order LL, OF, ML
        if (l == 0) out[p] = (uint8_t)((m_ll << 6) | (m_of << 4) | (m_ml << 2));
        for (uint32_t i = l; i < n_ll + n_of + n_ml; i += 64) {
            uint8_t v;
            if (i < n_ll) v = hz.nc[i];
            else if (i < n_ll + n_of) v = hz.nc[128 + i - n_ll];
            else v = hz.nc[64 + i - n_ll - n_of];
            out[p + 1 + i] = v;
        }
        p += 1 + n_ll + n_of + n_ml;
        wsync();
        // the bitstream: sequence nseq - 1 first; per sequence [OF st][ML st][LL st][LL x][ML x][OF x]
        const uint32_t base = 8 * p;
        uint32_t carry = 0;
        for (int c0 = (int)((nseq - 1) & ~63u); c0 >= 0; c0 -= 64) {
            const uint32_t n = (uint32_t)c0 + l;
            const bool v = n < nseq;
            uint32_t lit = 0, len = 0, obase = 1, llc = 0, mlc = 0;
            if (v) {
                const uint32_t s0 = seq[2 * n], w = seq[2 * n + 1];
                lit = s0 & 0xFFFF;
                len = s0 >> 16;
                obase = w & 0xFFFF;
                llc = (w >> 16) & 63;
                mlc = (w >> 22) & 63;
            }
            const uint32_t ofc = hibit(obase);
            const uint32_t llb = c_zll_bits[llc], mlb = c_zml_bits[mlc];
            uint32_t e_of = 0, e_ml = 0, e_ll = 0;
            if (v && n + 1 < nseq) {
                e_ll = fsei[n];
                e_ml = fsei[1024 + n];
                e_of = fsei[2048 + n];
            }
            const uint32_t nb_of = e_of >> 12, nb_ml = e_ml >> 12, nb_ll = e_ll >> 12;
            const uint32_t b = v ? nb_of + nb_ml + nb_ll + llb + mlb + ofc : 0;
            const uint32_t inc = wave_incl_scan(b), tot = wave_readlane(inc, 63);
            uint32_t pos = base + carry + (tot - inc);
            if (v) {
                put_bits(bw, pos, e_of & 0xFFF, nb_of);
                pos += nb_of;
                put_bits(bw, pos, e_ml & 0xFFF, nb_ml);
                pos += nb_ml;
                put_bits(bw, pos, e_ll & 0xFFF, nb_ll);
                pos += nb_ll;
                put_bits(bw, pos, lit - c_zll_base[llc], llb);
                pos += llb;
                put_bits(bw, pos, len - c_zml_base[mlc], mlb);
                pos += mlb;
                put_bits(bw, pos, obase - (1u << ofc), ofc);
            }
            carry += tot;
        }
        if (l == 0) {
            uint32_t pos = base + carry;
            put_bits(bw, pos, hz.misc[9], al_ml);
            pos += al_ml;
            put_bits(bw, pos, hz.misc[10], al_of);
            pos += al_of;
            put_bits(bw, pos, hz.misc[8], al_ll);
            pos += al_ll;
            put_bits(bw, pos, 1u, 1);
        }
        wsync();
        p += (carry + al_ml + al_of + al_ll) / 8 + 1;
    }
    wsync();
    const uint32_t content = p - ob;
    return content < wn ? content : 0;
}

// ------------------------------------------------------------------------------------------------
// C1: compress.  One wave per block, windows of <= 4 KiB.
// ------------------------------------------------------------------------------------------------
template <uint32_t CODEC>
__global__ __launch_bounds__(64 * CzCfg<CODEC>::kWaves) void k_cz(CzArgs a) {
    using Cfg = CzCfg<CODEC>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (lds_addr((const void *)smem) != 0) {
        if (threadIdx.x == 0) atomicMin(a.err, (unsigned long long)SDB_DEVICE_ERROR);
        return;
    }
    cz_crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    lu8 *wb = (lu8 *)smem + kCzCrcLds + w * Cfg::kWaveLds;
    lu8 *in = wb;
    lu32 *head = (lu32 *)(wb + kCzIn);
    lu32 *seq = head;  // after the match pass: 2 dwords per sequence
    lu16 *prev = (lu16 *)(wb + kCzIn + kCzHead);
    lu8 *hz = (lu8 *)prev;  // after the match pass: the entropy coders' scratch (zlib / zstd)
    lu32 *mm = (lu32 *)(wb + kCzIn + kCzHead + (Cfg::kDeep ? kCzPrev : 0));
    lu8 *out = (lu8 *)mm + kCzOutOff;
    lu8 *aux = (lu8 *)mm + kCzAuxOff;
    const uint64_t base = a.block_off[0];
    for (uint64_t k = (uint64_t)blockIdx.x * Cfg::kWaves + w; k < a.nblocks; k += (uint64_t)gridDim.x * Cfg::kWaves) {
        const uint64_t s = a.block_off[k], e = a.block_off[k + 1];
        if (e < s + 4 || e - base > a.in_bytes) {  // no block (Block::encode() ++ CRC is >= 8 bytes), or past in_bytes
            if (l == 0) {
                atomicMin(a.err, (unsigned long long)((k << 8) | (e < s + 4 ? SDB_CORRUPT_BLOCK : SDB_INVALID_ARGUMENT)));
                a.len[k] = 0;
            }
            continue;
        }
        uint8_t *slot = a.slots + cz_slot(s - base, k);
        const uint32_t n = (uint32_t)(e - 4 - s);  // Block::encode() bytes (the stored CRC is not compressed)
        const uint8_t *src = a.blocks + s;
        // window state (wave-uniform)
        uint32_t w0 = 0, opos = 0, crc = 0;
        uint32_t zcarry = 0, zbyte = 0;  // zlib: bits of a partial byte carried into the next window
        uint64_t sa = 0, sb = 0;         // zlib: Adler-32 sums
        uint32_t rep[3] = {1, 4, 8};     // zstd: repeat offsets
        bool fallback = false;
        CZ_T0(kt);
        for (;;) {
            const uint32_t wn = n - w0 < kCzWin ? n - w0 : kCzWin;
            const bool first = w0 == 0, last = w0 + wn == n;
            // stage the window (16-byte granules) and zero the 64 bytes past it
            {
                const uint64_t g0 = (s + w0) & ~15ull;
                const uint32_t lead = (uint32_t)(s + w0 - g0), ng = (lead + wn + 15) >> 4;
                for (uint32_t q = l; q < ng; q += 64) {
                    const uint4 v = ((const uint4 *)(a.blocks + g0))[q];
                    const uint32_t d0 = 16 * q;
                    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int b = 0; b < 16; b++) {
                        const int64_t x = (int64_t)d0 + b - lead;
                        if (x >= 0 && x < (int64_t)wn) in[x] = (uint8_t)(vv[b >> 2] >> (8 * (b & 3)));
                    }
                }
                in[wn + l] = 0;
            }
            wsync();
            CZ_MARK(0, kt);
            const uint64_t vmask = cz_matches<CODEC>(in, wn, n - w0, head, prev, mm);
            CZ_MARK(1, kt);
            uint32_t tail = 0;
            const uint32_t nseq = cz_parse(vmask, wn, mm, seq, &tail);
            CZ_MARK(2, kt);
            if (CODEC == SDB_CODEC_LZ4 && !last && nseq == 0) {  // no sequence can end this window
                fallback = true;
                break;
            }
            // c. the codec's elements into out (the mm region: its match words are no longer needed)
            for (uint32_t q = l; q < kCzOutCap / 4 + 16; q += 64) ((lu32 *)mm)[q] = 0;  // lead-in + out
            wsync();
            uint32_t m = 0;        // output bytes of this window
            uint32_t next_w0 = w0 + wn;
            if constexpr (CODEC == SDB_CODEC_ZSTD) {
                uint32_t hb = 0;
                if (first && l == 0) {
                    out[0] = 0x28; out[1] = 0xB5; out[2] = 0x2F; out[3] = 0xFD;
                    uint32_t p = 4;
                    if (n < 256) { out[p++] = 0x20; out[p++] = (uint8_t)n; }
                    else if (n < 65536 + 256) { out[p++] = 0x60; out[p++] = (uint8_t)(n - 256); out[p++] = (uint8_t)((n - 256) >> 8); }
                    else { out[p++] = 0xA0; out[p++] = (uint8_t)n; out[p++] = (uint8_t)(n >> 8); out[p++] = (uint8_t)(n >> 16); out[p++] = (uint8_t)(n >> 24); }
                }
                if (first) hb = n < 256 ? 6 : (n < 65536 + 256 ? 7 : 9);
                const uint8_t b0 = in[0];
                bool same = true;
                for (uint32_t i = l; i < wn; i += 64) same &= in[i] == b0;
                same = __ballot(!same) == 0 && wn > 0;
                uint32_t content = 0, btype = 0;
#ifdef SDB_CZ_NOENT  // diagnostic: raw blocks (the match pass and parse only)
                if (false) {
#else
                if (!same && wn >= 16) {
#endif
                    content = cz_zstd_window(in, wn, seq, nseq, out, hb + 3, rep, hz, aux);
                    btype = content ? 2 : 0;
                } else if (same) {
                    btype = 1;
                }
                if (btype == 0) {  // raw block: the window's bytes (the bit region may hold a discarded attempt)
                    for (uint32_t i = l; i < wn; i += 64) out[hb + 3 + i] = in[i];
                    content = wn;
                } else if (btype == 1) {
                    if (l == 0) out[hb + 3] = b0;
                    content = 1;
                }
                if (l == 0) {
                    const uint32_t bh = (last ? 1u : 0u) | (btype << 1) | ((btype == 1 ? wn : content) << 3);
                    out[hb] = (uint8_t)bh; out[hb + 1] = (uint8_t)(bh >> 8); out[hb + 2] = (uint8_t)(bh >> 16);
                }
                m = hb + 3 + content;
                // the rest of the bit region past m is never read: the slot copy takes [0, m)
            } else if constexpr (CODEC == SDB_CODEC_ZLIB) {
                uint32_t hb = 0;
                if (first && l == 0) {
                    out[0] = 0x78;
                    out[1] = 0x9C;
                }
                if (first) hb = 2;
                else if (l == 0 && zcarry) out[0] = (uint8_t)zbyte;
                wsync();
                {
                    uint64_t xa = 0, xb = 0;
                    for (uint32_t i = l; i < wn; i += 64) {
                        xa += in[i];
                        xb += (uint64_t)(n - (w0 + i)) * in[i];
                    }
                    sa += wave_sum(xa);
                    sb += wave_sum(xb);
                }
                const uint32_t endb = cz_deflate_window(in, wn, seq, nseq, out, 8 * hb + zcarry, last, hz, aux);
                if (last) {
                    m = (endb + 7) >> 3;
                    const uint32_t A = (uint32_t)((1 + sa) % 65521), B = (uint32_t)((n + sb) % 65521);
                    if (l == 0) {
                        out[m] = (uint8_t)(B >> 8); out[m + 1] = (uint8_t)B; out[m + 2] = (uint8_t)(A >> 8); out[m + 3] = (uint8_t)A;
                    }
                    m += 4;
                } else {
                    m = endb >> 3;
                    zcarry = endb & 7;
                    zbyte = zcarry ? out[m] : 0;
                }
            } else {
                // LZ4 / Snappy: byte elements.  Header: lz4 u32 LE length; snappy varint length.
                uint32_t hdr = 0;
                if (first) hdr = CODEC == SDB_CODEC_LZ4 ? 4 : (n < 128 ? 1 : (n < 16384 ? 2 : (n < (1u << 21) ? 3 : 4)));
                if (first && l == 0) {
                    if (CODEC == SDB_CODEC_LZ4) {
                        out[0] = (uint8_t)n; out[1] = (uint8_t)(n >> 8); out[2] = (uint8_t)(n >> 16); out[3] = (uint8_t)(n >> 24);
                    } else {
                        uint32_t x = n, p = 0;
                        for (;; x >>= 7) {
                            out[p++] = (uint8_t)(x >= 0x80 ? (x & 0x7F) | 0x80 : x);
                            if (x < 0x80) break;
                        }
                    }
                }
                auto lit_hdr = [](uint32_t lit) -> uint32_t {
                    if (CODEC == SDB_CODEC_LZ4) return lit >= 15 ? (lit - 15) / 255 + 1 : 0;  // (the token counted with the match)
                    if (!lit) return 0;
                    const uint32_t v = lit - 1;
                    return v < 60 ? 1 : v < 256 ? 2 : 3;
                };
                auto match_bytes = [](uint32_t len, uint32_t off) -> uint32_t {
                    if (CODEC == SDB_CODEC_LZ4) return 2 + (len - 4 >= 15 ? (len - 4 - 15) / 255 + 1 : 0);
                    uint32_t b = 0;  // snappy: copy-2 elements of 64 (60 before a short tail), then the rest
                    while (len >= 68) { b += 3; len -= 64; }
                    if (len > 64) { b += 3; len -= 60; }
                    return b + ((len < 12 && off < 2048) ? 2 : 3);
                };
                const uint32_t nchunk = (nseq + 63) / 64;
                uint32_t carry_out = hdr, carry_pos = 0;
                for (uint32_t ch = 0; ch < nchunk; ch++) {
                    const uint32_t i = 64 * ch + l;
                    const bool v = i < nseq;
                    const uint32_t s0 = v ? seq[2 * i] : 0, off = v ? seq[2 * i + 1] : 0;
                    const uint32_t lit = s0 & 0xFFFF, len = s0 >> 16;
                    const uint32_t span = lit + len, pinc = wave_incl_scan(span);
                    const uint32_t lstart = carry_pos + pinc - span;
                    const uint32_t lh = v ? lit_hdr(lit) : 0, mb = v ? match_bytes(len, off) : 0;
                    const uint32_t sz = v ? (CODEC == SDB_CODEC_LZ4 ? 1 : 0) + lh + lit + mb : 0;
                    const uint32_t oinc = wave_incl_scan(sz);
                    const uint32_t o0 = carry_out + oinc - sz;
                    if (v) {
                        uint32_t p = o0;
                        if (CODEC == SDB_CODEC_LZ4) {
                            const uint32_t ml = len - 4;
                            out[p++] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (ml >= 15 ? 15 : ml));
                            if (lit >= 15) {
                                uint32_t x = lit - 15;
                                for (; x >= 255; x -= 255) out[p++] = 255;
                                out[p++] = (uint8_t)x;
                            }
                            p += lit;
                            out[p++] = (uint8_t)off;
                            out[p++] = (uint8_t)(off >> 8);
                            if (ml >= 15) {
                                uint32_t x = ml - 15;
                                for (; x >= 255; x -= 255) out[p++] = 255;
                                out[p++] = (uint8_t)x;
                            }
                        } else {
                            if (lit) {
                                const uint32_t x = lit - 1;
                                if (x < 60) out[p++] = (uint8_t)(x << 2);
                                else if (x < 256) { out[p++] = 60 << 2; out[p++] = (uint8_t)x; }
                                else { out[p++] = 61 << 2; out[p++] = (uint8_t)x; out[p++] = (uint8_t)(x >> 8); }
                            }
                            p += lit;
                            uint32_t r = len;
                            auto copy2 = [&](uint32_t c) {
                                out[p++] = (uint8_t)(2 | ((c - 1) << 2));
                                out[p++] = (uint8_t)off;
                                out[p++] = (uint8_t)(off >> 8);
                            };
                            while (r >= 68) { copy2(64); r -= 64; }
                            if (r > 64) { copy2(60); r -= 60; }
                            if (r < 12 && off < 2048) {
                                out[p++] = (uint8_t)(1 | ((r - 4) << 2) | ((off >> 8) << 5));
                                out[p++] = (uint8_t)off;
                            } else {
                                copy2(r);
                            }
                        }
                    }
                    // the chunk's literal runs, by the wave
                    const uint32_t lpos = o0 + (CODEC == SDB_CODEC_LZ4 ? 1 : 0) + lh;
                    const uint32_t ncur = nseq - 64 * ch < 64 ? nseq - 64 * ch : 64;
                    for (uint32_t j = 0; j < ncur; j++) {
                        const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)lstart, (int)j);
                        const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane((int)lit, (int)j);
                        const uint32_t dst = (uint32_t)__builtin_amdgcn_readlane((int)lpos, (int)j);
                        for (uint32_t x = l; x < cnt; x += 64) out[dst + x] = in[sj + x];
                    }
                    carry_out += wave_readlane(oinc, 63);
                    carry_pos += wave_readlane(pinc, 63);
                }
                // the window's final literals (lz4: only in the last window, as its last sequence; the
                // other windows end at their last match and the next window starts there)
                if (CODEC == SDB_CODEC_LZ4 && !last) {
                    m = carry_out;
                    next_w0 = w0 + tail;
                } else {
                    const uint32_t lit = wn - carry_pos;
                    uint32_t p = carry_out;
                    if (CODEC == SDB_CODEC_LZ4) {
                        if (l == 0) {
                            out[p] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
                            if (lit >= 15) {
                                uint32_t x = lit - 15, q = p + 1;
                                for (; x >= 255; x -= 255) out[q++] = 255;
                                out[q] = (uint8_t)x;
                            }
                        }
                        p += 1 + lit_hdr(lit);
                    } else if (lit) {
                        if (l == 0) {
                            const uint32_t x = lit - 1;
                            if (x < 60) out[p] = (uint8_t)(x << 2);
                            else if (x < 256) { out[p] = 60 << 2; out[p + 1] = (uint8_t)x; }
                            else { out[p] = 61 << 2; out[p + 1] = (uint8_t)x; out[p + 2] = (uint8_t)(x >> 8); }
                        }
                        p += lit_hdr(lit);
                    }
                    for (uint32_t x = l; x < lit; x += 64) out[p + x] = in[carry_pos + x];
                    m = p + lit;
                }
            }
            wsync();
            CZ_MARK(3, kt);
            // d. CRC32 of the window's bytes (chained), then the slot
            if (l < 16) ((lu32 *)mm)[l] = 0;  // the lead-in (scratch above may have used it)
            wsync();
            const uint32_t raw = cz_crc_raw(out, m, aux + 64, first);
            crc = crc_shift_bytes(crc, m) ^ raw;
            if (first && last) {  // one window: the CRC after the bytes, 16-byte stores into the aligned slot
                const uint32_t c = ~crc;
                if (l == 0) {
                    out[m] = (uint8_t)(c >> 24); out[m + 1] = (uint8_t)(c >> 16); out[m + 2] = (uint8_t)(c >> 8); out[m + 3] = (uint8_t)c;
                    a.len[k] = m + 4;
                }
                wsync();
                const uint32_t n16 = (m + 4 + 15) >> 4;
                for (uint32_t q = l; q < n16; q += 64) {
                    const u32x4 v = ((const lu128 *)out)[q];
                    uint4 g;
                    g.x = v.x;
                    g.y = v.y;
                    g.z = v.z;
                    g.w = v.w;
                    ((uint4 *)slot)[q] = g;
                }
                wsync();
                CZ_MARK(4, kt);
                break;
            }
            CZ_MARK(4, kt);
            for (uint32_t i = l; i < m; i += 64) slot[opos + i] = out[i];
            opos += m;
            wsync();
            if (last) {
                const uint32_t c = ~crc;
                if (l < 4) slot[opos + l] = (uint8_t)(c >> (24 - 8 * l));
                if (l == 0) a.len[k] = opos + 4;
                break;
            }
            w0 = next_w0;
        }
        if (fallback && l == 0) {  // lz4 only: one literal-only sequence, by one lane
            const uint32_t m = cz_literal_only(CODEC, src, n, slot);
            uint32_t c = 0xFFFFFFFFu;
            for (uint32_t i = 0; i < m; i++) c = (c >> 8) ^ c_crc.t[0][(c ^ slot[i]) & 0xFF];
            c = ~c;
            slot[m] = (uint8_t)(c >> 24); slot[m + 1] = (uint8_t)(c >> 16); slot[m + 2] = (uint8_t)(c >> 8); slot[m + 3] = (uint8_t)c;
            a.len[k] = m + 4;
        }
        wsync();
    }
}

// C3: slot k -> out[out_off[k], out_off[k + 1])
__global__ __launch_bounds__(256) void k_cz_pack(CzArgs a) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t total = a.out_off[a.nblocks];
    if (total > a.out_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicMin(a.err, (unsigned long long)((a.nblocks << 8) | SDB_LIMIT_EXCEEDED));
        return;
    }
    const uint64_t base = a.block_off[0];
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); k < a.nblocks; k += nw) {
        const uint8_t *src = a.slots + cz_slot(a.block_off[k] - base, k);
        uint8_t *dst = a.out + a.out_off[k];
        const uint64_t len = a.out_off[k + 1] - a.out_off[k];
        // bytes up to the destination's first 16-byte boundary, then 16-byte stores of realigned source
        // bytes (unaligned 16-byte loads), then the tail
        const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15) < len ? (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15) : (uint32_t)len;
        if (l < head) dst[l] = src[l];
        const uint64_t body = (len - head) & ~15ull;
        for (uint64_t q = l; q < body / 16; q += 64) {
            uint4 v;
            __builtin_memcpy(&v, src + head + 16 * q, 16);
            *(uint4 *)(dst + head + 16 * q) = v;
        }
        for (uint64_t i = head + body + l; i < len; i += 64) dst[i] = src[i];
    }
}

extern "C" int sdb_diag_cz_phase(uint64_t *out, int reset) {  // -DSDB_CZ_PT builds: ticks per phase
#ifdef SDB_CZ_PT
    if (reset) {
        static const unsigned long long z[16] = {};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_cz_pt), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cz_pt), 16 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
#else
    (void)out;
    (void)reset;
    return -1;
#endif
}

static std::once_flag g_cz_once;

uint64_t compress_workspace_bytes(uint64_t nblocks, uint64_t in_bytes) {
    const uint64_t slots = cz_slot(in_bytes, nblocks) + 256;
    const uint64_t nt = (nblocks + 1023) / 1024 + 1;
    return slots + 8 * (nblocks + 2) * 2 + 16 * (nt + 1) + 512;
}

template <uint32_t C>
static void cz_launch(const CzArgs &a, hipStream_t st) {
    using Cfg = CzCfg<C>;
    const uint64_t wgs = (a.nblocks + Cfg::kWaves - 1) / Cfg::kWaves;
    const uint32_t grid = (uint32_t)(wgs < 4096 ? wgs : 4096);
    hipLaunchKernelGGL(k_cz<C>, dim3(grid), dim3(64 * Cfg::kWaves), Cfg::kLds, st, a);
}

hipError_t launch_compress(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                           uint64_t in_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                           unsigned long long *err, void *ws, hipStream_t st) {
    std::call_once(g_cz_once, [] {
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_LZ4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CzCfg<SDB_CODEC_LZ4>::kLds);
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_SNAPPY>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CzCfg<SDB_CODEC_SNAPPY>::kLds);
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_ZLIB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CzCfg<SDB_CODEC_ZLIB>::kLds);
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_ZSTD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CzCfg<SDB_CODEC_ZSTD>::kLds);
        (void)hipGetLastError();
    });
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    CzArgs a{};
    a.codec = codec;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.in_bytes = in_bytes;
    a.slots = w;
    uint8_t *tail = w + ((cz_slot(in_bytes, nblocks) + 255) & ~255ull);
    a.len = (uint64_t *)tail;
    uint64_t *scratch = a.len + (nblocks + 2);
    const uint64_t nt = (nblocks + 1023) / 1024 + 1;
    uint64_t *tx = scratch + (nblocks + 2), *ty = tx + (nt + 1);
    a.out = out;
    a.out_cap = out_cap;
    a.out_off = out_off;
    a.err = err;
    if (hipMemsetAsync(err, 0xFF, 8, st) != hipSuccess) return hipErrorUnknown;
    if (!nblocks) return hipMemsetAsync(out_off, 0, 8, st);
    switch (codec) {
        case SDB_CODEC_LZ4: cz_launch<SDB_CODEC_LZ4>(a, st); break;
        case SDB_CODEC_SNAPPY: cz_launch<SDB_CODEC_SNAPPY>(a, st); break;
        case SDB_CODEC_ZLIB: cz_launch<SDB_CODEC_ZLIB>(a, st); break;
        default: cz_launch<SDB_CODEC_ZSTD>(a, st); break;
    }
    hipError_t e = launch_excl_scan2(a.len, a.len, nblocks, tx, ty, out_off, scratch, st);
    if (e != hipSuccess) return e;
    const uint32_t pgrid = (uint32_t)((nblocks + 3) / 4 < 4096 ? (nblocks + 3) / 4 : 4096);
    hipLaunchKernelGGL(k_cz_pack, dim3(pgrid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace sdb
