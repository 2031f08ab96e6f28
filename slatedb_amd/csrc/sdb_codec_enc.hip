// sdb_codec_enc.hip — the compressing write side of SURVEY §8(f) row f3 for gfx950.
//
// Replaces compress_and_transform (slatedb/src/format/sst.rs:525-554) with SsTableFormat::compress
// (format/sst.rs:557-594) for every block of an encoded data section: the codec's bytes of
// Block::encode(), then the CRC32 (BE) of those compressed bytes:
//   Lz4    lz4_flex 0.11.6 block::compress_prepend_size: u32 LE length ++ one LZ4 block;
//   Snappy snap 1.1.1 raw::Encoder::compress_vec: varint length ++ Snappy raw elements;
//   Zlib   flate2 1.1.9 ZlibEncoder (default level): 78 9C ++ deflate ++ Adler-32 BE;
//   Zstd   zstd 0.13.3 bulk::compress(data, 3): one frame with Frame_Content_Size (single segment).
// A compressor's output bytes are a choice of its match finder, not of the format: these streams are
// valid for the formats (they decode through the reference's decompressors — and sdb_decompress_blocks,
// the oracle, pyarrow / zlib in the tests — to the same block bytes) but are not the crates' bytes.
//
//   C1 compress  one wave per block (four per workgroup, the block in the wave's LDS):
//                a. every position's match: a 4-byte hash into a 2048-entry table of the latest earlier
//                   position (built 64 positions at a time: each lane reads its bucket, then the batch
//                   stores its positions with ds_max_u32), verified and extended bytewise (<= 258);
//                b. the greedy parse: one wave-uniform walk over the chosen matches only (lane w holds the
//                   match bitmap of positions [64 w, 64 w + 64): the next match is one ballot away), the
//                   sequences (literal run, offset, length) listed in LDS;
//                c. the codec's elements: lanes size their sequence's elements, a wave scan places them,
//                   each lane writes its headers / match codes and the wave copies the literal runs;
//                   deflate as fixed-Huffman codes (bit positions from a prefix count of the literals
//                   that take 9 bits) or a stored block when that is shorter; zstd as one raw (or RLE)
//                   block;
//                d. the wave CRC32 of the compressed bytes (two windows past 4 KiB), the slot written to
//                   the workspace, its length recorded.
//                Blocks over 4 KiB (SstBlockSize 8-64 KiB) are written by one lane as literal-only
//                streams (stored deflate, raw zstd).
//   C2 scan      exclusive scan of the lengths -> out_off (the compressed BlockMeta offsets).
//   C3 pack      one wave per block: slot -> out[out_off[k], out_off[k+1]).
#include <mutex>

#include "sdb_crc.h"
#include "sdb_decode.h"
#include "sdb_device.h"

namespace sdb {

typedef __attribute__((address_space(3))) uint16_t lu16;

constexpr uint32_t kCzWaves = 4, kCzThreads = 64 * kCzWaves;
constexpr uint32_t kCzMax = 4096;              // fast path: blocks of at most 4 KiB
constexpr uint32_t kCzHashBits = 11;
constexpr uint32_t kCzIn = kCzMax + 64;        // the block (+ zeros for reads past its end)
constexpr uint32_t kCzHt = 4u << kCzHashBits;  // hash table (u32 position + 1), then the sequence list
constexpr uint32_t kCzMm = 4 * kCzMax;         // per position off << 16 | len; then the output (at +64) and
                                               // zlib's prefix count of 9-bit literals (at +8 KiB)
constexpr uint32_t kCzWaveLds = kCzIn + kCzHt + kCzMm + 64 * 8;
constexpr uint32_t kCzLds = kCrcTablesLds + kCzWaves * kCzWaveLds;
static_assert(kCzLds <= 160 * 1024, "compress LDS");
constexpr uint32_t kCzMaxSeq = kCzHt / 8 - 8;  // sequences listed per block (the rest stays literal)
constexpr uint32_t kCzOutOff = 64;             // the output at mm + 64: the CRC's 64 zero lead-in bytes before it
constexpr uint32_t kCzP9Off = 8192;
constexpr uint32_t kCzMaxMatch = 258;

// block k's slot in the workspace (rel = block_off[k] - block_off[0]): compressed bytes + CRC stay under
// n + n/8 + 48 for every codec here (literal-only worst cases: lz4 n + n/255 + 10, snappy n + 14, stored
// deflate n + 15, raw zstd n + 16)
__host__ __device__ inline uint64_t cz_slot(uint64_t rel, uint64_t k) { return (rel + rel / 8 + 64 * k + 15) & ~15ull; }

struct CzArgs {
    uint32_t codec;
    const uint8_t *blocks;
    const uint64_t *block_off;  // nblocks + 1
    uint64_t nblocks;
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
SDB_DEV uint32_t cz_hash(uint32_t v) { return (v * 2654435761u) >> (32 - kCzHashBits); }

// deflate's fixed Huffman code (RFC 1951 3.2.6) of a literal / length symbol, bit-reversed for the
// LSB-first stream: value in the low `*nb` bits
SDB_DEV uint32_t rev_bits(uint32_t v, uint32_t n) { return __builtin_bitreverse32(v) >> (32 - n); }
SDB_DEV uint32_t fixed_code(uint32_t sym, uint32_t *nb) {
    if (sym < 144) { *nb = 8; return rev_bits(0x30 + sym, 8); }
    if (sym < 256) { *nb = 9; return rev_bits(0x190 + sym - 144, 9); }
    if (sym < 280) { *nb = 7; return rev_bits(sym - 256, 7); }
    *nb = 8;
    return rev_bits(0xC0 + sym - 280, 8);
}
__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
// a match (len 3..258, dist 1..32768) as fixed-Huffman bits: up to 7 + 5 + 5 + 13 = 30 bits (one u32)
SDB_DEV uint32_t deflate_match(uint32_t len, uint32_t dist, uint32_t *nb) {
    uint32_t lc = 0;
    while (lc < 28 && c_len_base[lc + 1] <= len) lc++;
    uint32_t dc = 0;
    while (dc < 29 && c_dist_base[dc + 1] <= dist) dc++;
    uint32_t n0;
    uint32_t v = fixed_code(257 + lc, &n0), n = n0;
    v |= (len - c_len_base[lc]) << n;
    n += c_len_extra[lc];
    v |= rev_bits(dc, 5) << n;
    n += 5;
    v |= (dist - c_dist_base[dc]) << n;
    n += c_dist_extra[dc];
    *nb = n;
    return v;
}

// OR `nb` (<= 32) bits `v` into the LDS bitstream `w` (u32 words, zeroed) at bit position `pos`
SDB_DEV void put_bits(lu32 *w, uint32_t pos, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t q = pos >> 5, r = pos & 31;
    __hip_atomic_fetch_or(&w[q], v << r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (r + nb > 32) __hip_atomic_fetch_or(&w[q + 1], v >> (32 - r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// crc32fast::hash of out[0, m), m <= 4096 + 1024, by the wave (out 16-byte aligned, the 64 bytes before it
// zero): [0, min(m, 4096)) in place, the rest (when m > 4096) copied to `sc` (16-byte aligned, 64 free bytes
// before it), combined by x^(8 (m - 4096))
SDB_DEV void wsync();
SDB_DEV uint32_t cz_crc(lu8 *out, uint32_t m, lu8 *sc) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t head = m > 4096 ? 4096 : m, tail = m - head;
    if (tail) {
        if (l < 16) ((lu32 *)(sc - 64))[l] = 0;
        for (uint32_t i = l; i < tail; i += 64) sc[i] = out[4096 + i];
    }
    if (l == 0) ((lu32 *)out)[0] = ~((const lu32 *)out)[0];  // crc32fast's init, folded into bytes [0, 4)
    wsync();
    uint32_t raw = wave_crc_image_ra(out, head) ^ 0xFFFFFFFFu;
    if (tail) raw = crc_shift_bytes(raw, tail) ^ wave_crc_image_ra(sc, tail) ^ 0xFFFFFFFFu;
    wsync();
    if (l == 0) ((lu32 *)out)[0] = ~((const lu32 *)out)[0];
    wsync();
    return raw ^ 0xFFFFFFFFu;
}

SDB_DEV void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------------------------------------
// One lane, any size: a literal-only stream of the codec straight into the global slot (blocks over
// the wave's LDS).  Returns the bytes written (without the CRC).
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
    } else if (codec == SDB_CODEC_SNAPPY) {
        for (uint32_t x = n;; x >>= 7) {
            o[p++] = (uint8_t)(x >= 0x80 ? (x & 0x7F) | 0x80 : x);
            if (x < 0x80) break;
        }
        if (n) {
            const uint32_t v = n - 1;
            if (v < 60) o[p++] = (uint8_t)(v << 2);
            else if (v < 256) { o[p++] = 60 << 2; o[p++] = (uint8_t)v; }
            else if (v < 65536) { o[p++] = 61 << 2; o[p++] = (uint8_t)v; o[p++] = (uint8_t)(v >> 8); }
            else if (v < (1u << 24)) { o[p++] = 62 << 2; o[p++] = (uint8_t)v; o[p++] = (uint8_t)(v >> 8); o[p++] = (uint8_t)(v >> 16); }
            else { o[p++] = 63 << 2; o[p++] = (uint8_t)v; o[p++] = (uint8_t)(v >> 8); o[p++] = (uint8_t)(v >> 16); o[p++] = (uint8_t)(v >> 24); }
            lit_copy(in, n);
        }
    } else if (codec == SDB_CODEC_ZLIB) {
        o[p++] = 0x78;
        o[p++] = 0x9C;
        uint32_t a = 1, b = 0;
        for (uint32_t i = 0; i < n; i++) {
            a += in[i];
            if (a >= 65521) a -= 65521;
            b += a;
            if (b >= 65521) b -= 65521;
        }
        uint32_t done = 0;
        do {  // stored blocks of <= 65535 bytes
            const uint32_t c = n - done < 65535 ? n - done : 65535;
            o[p++] = done + c == n ? 1 : 0;
            o[p++] = (uint8_t)c; o[p++] = (uint8_t)(c >> 8);
            o[p++] = (uint8_t)~c; o[p++] = (uint8_t)(~c >> 8);
            lit_copy(in + done, c);
            done += c;
        } while (done < n);
        o[p++] = (uint8_t)(b >> 8); o[p++] = (uint8_t)b; o[p++] = (uint8_t)(a >> 8); o[p++] = (uint8_t)a;
    } else {  // zstd: one frame, raw blocks of <= 128 KiB
        o[0] = 0x28; o[1] = 0xB5; o[2] = 0x2F; o[3] = 0xFD;
        p = 4;
        if (n < 256) { o[p++] = 0x20; o[p++] = (uint8_t)n; }
        else if (n < 65536 + 256) { o[p++] = 0x60; o[p++] = (uint8_t)(n - 256); o[p++] = (uint8_t)((n - 256) >> 8); }
        else { o[p++] = 0xA0; o[p++] = (uint8_t)n; o[p++] = (uint8_t)(n >> 8); o[p++] = (uint8_t)(n >> 16); o[p++] = (uint8_t)(n >> 24); }
        uint32_t done = 0;
        do {
            const uint32_t c = n - done < (128u << 10) ? n - done : (128u << 10);
            const uint32_t bh = (done + c == n ? 1u : 0u) | (c << 3);  // Raw_Block
            o[p++] = (uint8_t)bh; o[p++] = (uint8_t)(bh >> 8); o[p++] = (uint8_t)(bh >> 16);
            lit_copy(in + done, c);
            done += c;
        } while (done < n);
    }
    return p;
}

// ------------------------------------------------------------------------------------------------
// C1: compress.  Lane l of a wave owns: positions l, l + 64, ... in the match pass; sequence l of each
// 64-sequence chunk in the element pass.
// ------------------------------------------------------------------------------------------------
template <uint32_t CODEC>
__global__ __launch_bounds__(kCzThreads) void k_cz(CzArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (lds_addr((const void *)smem) != 0) {
        if (threadIdx.x == 0) atomicMin(a.err, (unsigned long long)SDB_DEVICE_ERROR);
        return;
    }
    crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    lu8 *wb = (lu8 *)smem + kCrcTablesLds + w * kCzWaveLds;
    lu8 *in = wb;
    lu32 *ht = (lu32 *)(wb + kCzIn);
    lu32 *seq = ht;  // after the match pass: 2 dwords per sequence (lit | mlen << 16, off)
    lu32 *mm = (lu32 *)(wb + kCzIn + kCzHt);
    lu8 *out = (lu8 *)mm + kCzOutOff;
    lu16 *p9 = (lu16 *)((lu8 *)mm + kCzP9Off);
    const uint64_t base = a.block_off[0];
    for (uint64_t k = (uint64_t)blockIdx.x * kCzWaves + w; k < a.nblocks; k += (uint64_t)gridDim.x * kCzWaves) {
        const uint64_t s = a.block_off[k], e = a.block_off[k + 1];
        uint8_t *slot = a.slots + cz_slot(s - base, k);
        if (e < s + 4) {  // no block (Block::encode() ++ CRC is at least 8 bytes): the caller's error
            if (l == 0) {
                atomicMin(a.err, (unsigned long long)((k << 8) | SDB_CORRUPT_BLOCK));
                a.len[k] = 0;
            }
            continue;
        }
        const uint32_t n = (uint32_t)(e - 4 - s);  // Block::encode() bytes (the stored CRC is not compressed)
        if (n > kCzMax) {
            uint32_t m = 0;
            if (l == 0) {
                m = cz_literal_only(CODEC, a.blocks + s, n, slot);
                uint32_t c = 0xFFFFFFFFu;
                for (uint32_t i = 0; i < m; i++) c = (c >> 8) ^ c_crc.t[0][(c ^ slot[i]) & 0xFF];
                c = ~c;
                slot[m] = (uint8_t)(c >> 24); slot[m + 1] = (uint8_t)(c >> 16); slot[m + 2] = (uint8_t)(c >> 8); slot[m + 3] = (uint8_t)c;
                a.len[k] = m + 4;
            }
            continue;
        }
        // stage the block (16-byte granules) and zero the 64 bytes past it
        {
            const uint64_t g0 = s & ~15ull;
            const uint32_t lead = (uint32_t)(s - g0), ng = (lead + n + 15) >> 4;
            for (uint32_t q = l; q < ng; q += 64) {
                const uint4 v = ((const uint4 *)(a.blocks + g0))[q];
                const uint32_t d0 = 16 * q;  // byte d0 - lead of the block
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int b = 0; b < 16; b++) {
                    const int64_t x = (int64_t)d0 + b - lead;
                    if (x >= 0 && x < (int64_t)n) in[x] = (uint8_t)(vv[b >> 2] >> (8 * (b & 3)));
                }
            }
            in[n + l] = 0;
            for (uint32_t q = l; q < (1u << kCzHashBits); q += 64) ht[q] = 0;
        }
        wsync();
        // a. matches: batches of 64 positions, lane = position
        uint64_t vmask = 0;
        const uint32_t last = n >= 4 ? n - 4 : 0;  // positions with 4 bytes to hash: [0, last]
        for (uint32_t b0 = 0; b0 <= last && n >= 4; b0 += 64) {
            const uint32_t p = b0 + l;
            const bool live = p <= last;
            const uint32_t v = live ? lds_u32u(in, p) : 0, h = cz_hash(v);
            const uint32_t cand = live ? ht[h] : 0;  // latest position + 1 of an earlier batch
            wsync();
            if (live) __hip_atomic_fetch_max(&ht[h], p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            uint32_t len = 0;
            const uint32_t q = cand - 1;
            if (live && cand && lds_u32u(in, q) == v) {
                len = 4;
                const uint32_t lim = n - p < kCzMaxMatch ? n - p : kCzMaxMatch;
                while (len < lim && in[q + len] == in[p + len]) len++;
            }
            if (CODEC == SDB_CODEC_LZ4) {  // LZ4: a match starts 12+ bytes before the end, ends 5+ before it
                if (p + 12 > n) len = 0;
                else if (len > n - 5 - p) len = n - 5 - p;
            }
            if (len < 4) len = 0;
            if (live) mm[p] = ((p - q) << 16) | len;
            const uint64_t bits = __ballot(len >= 4);
            if (l == (b0 >> 6)) vmask = bits;
            wsync();
        }
        // b. the greedy parse: lit_start / cur wave-uniform, the next match = first set bit >= cur
        uint32_t nseq = 0, ls = 0;
        {
            uint32_t cur = 0;
            while (nseq < kCzMaxSeq && cur < n) {
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
                if (l == 0) {
                    seq[2 * nseq] = (q - ls) | (len << 16);
                    seq[2 * nseq + 1] = off;
                }
                nseq++;
                ls = cur = q + len;
            }
        }
        wsync();
        // c. the codec's elements into out (the mm region: its match words are no longer needed)
        uint32_t m = 0;  // output bytes
        if (CODEC == SDB_CODEC_ZSTD) {
            // one frame, Single_Segment, Frame_Content_Size; one raw block (RLE when every byte is equal)
            const uint8_t b0 = in[0];
            bool same = true;
            for (uint32_t i = l; i < n; i += 64) same &= in[i] == b0;
            same = __ballot(!same) == 0 && n > 0;
            if (l == 0) {
                out[0] = 0x28; out[1] = 0xB5; out[2] = 0x2F; out[3] = 0xFD;
                uint32_t p = 4;
                if (n < 256) { out[p++] = 0x20; out[p++] = (uint8_t)n; }
                else { out[p++] = 0x60; out[p++] = (uint8_t)(n - 256); out[p++] = (uint8_t)((n - 256) >> 8); }
                const uint32_t bh = 1u | ((same ? 1u : 0u) << 1) | (n << 3);
                out[p++] = (uint8_t)bh; out[p++] = (uint8_t)(bh >> 8); out[p++] = (uint8_t)(bh >> 16);
                ((lu32 *)mm)[0] = p;  // (scratch: the header length, in the lead-in, re-zeroed below)
            }
            wsync();
            const uint32_t hdr = ((lu32 *)mm)[0];
            wsync();
            if (same) {
                if (l == 0) out[hdr] = b0;
                m = hdr + 1;
            } else {
                for (uint32_t i = l; i < n; i += 64) out[hdr + i] = in[i];
                m = hdr + n;
            }
        } else if (CODEC == SDB_CODEC_ZLIB) {
            // P9 = prefix count of literals >= 144 (9-bit codes), by 64-byte chunks with a carry
            {
                uint32_t carry = 0;
                for (uint32_t c0 = 0; c0 < n + 1; c0 += 64) {
                    const uint32_t i = c0 + l;
                    const uint32_t v = (i < n && in[i] >= 144) ? 1u : 0u;
                    const uint32_t inc = wave_incl_scan(v);
                    if (i <= n) p9[i] = (uint16_t)(carry + inc - v);
                    carry += wave_readlane(inc, 63);
                }
            }
            wsync();
            // sizes in bits: per sequence its literals + its match; the final literals after them
            const uint32_t nchunk = (nseq + 63) / 64;
            uint32_t carry_bits = 3, carry_pos = 0;  // after BFINAL / BTYPE
            lu32 *bw = (lu32 *)(out + 4);  // the deflate stream: 16-byte aligned words past the 2 header bytes + 2 pad
            // (out[2..4) pad: deflate bytes are gathered to out + 2 after the stream is complete)
            const uint32_t cap_words = (kCzP9Off - kCzOutOff - 8) / 4;
            for (uint32_t q = l; q < cap_words; q += 64) bw[q] = 0;
            wsync();
            if (l == 0) put_bits(bw, 0, 3, 3);  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
            for (uint32_t ch = 0; ch < nchunk; ch++) {
                const uint32_t i = 64 * ch + l;
                const bool v = i < nseq;
                const uint32_t s0 = v ? seq[2 * i] : 0, off = v ? seq[2 * i + 1] : 0;
                const uint32_t lit = s0 & 0xFFFF, len = s0 >> 16;
                const uint32_t span = lit + len;
                const uint32_t pinc = wave_incl_scan(span);
                const uint32_t lstart = carry_pos + pinc - span;
                uint32_t mb = 0, mbits = 0;
                if (v) mbits = deflate_match(len, off, &mb);
                const uint32_t bits = v ? 8 * lit + (p9[lstart + lit] - p9[lstart]) + mb : 0;
                const uint32_t binc = wave_incl_scan(bits);
                const uint32_t bstart = carry_bits + binc - bits;
                if (v) put_bits(bw, bstart + bits - mb, mbits, mb);
                // the chunk's literals, a sequence at a time, by the wave
                for (uint32_t j = 0; j < 64 && 64 * ch + j < nseq; j++) {
                    const uint32_t ls_j = (uint32_t)__builtin_amdgcn_readlane((int)lstart, (int)j);
                    const uint32_t lit_j = (uint32_t)__builtin_amdgcn_readlane((int)lit, (int)j);
                    const uint32_t b_j = (uint32_t)__builtin_amdgcn_readlane((int)bstart, (int)j);
                    for (uint32_t x = l; x < lit_j; x += 64) {
                        const uint32_t c = in[ls_j + x];
                        uint32_t nb;
                        const uint32_t code = fixed_code(c, &nb);
                        put_bits(bw, b_j + 8 * x + (p9[ls_j + x] - p9[ls_j]), code, nb);
                    }
                }
                carry_bits += wave_readlane(binc, 63);
                carry_pos += wave_readlane(pinc, 63);
            }
            // final literals [carry_pos, n), then end-of-block
            {
                const uint32_t ls_f = carry_pos, lit_f = n - carry_pos;
                for (uint32_t x = l; x < lit_f; x += 64) {
                    const uint32_t c = in[ls_f + x];
                    uint32_t nb;
                    const uint32_t code = fixed_code(c, &nb);
                    put_bits(bw, carry_bits + 8 * x + (p9[ls_f + x] - p9[ls_f]), code, nb);
                }
                carry_bits += 8 * lit_f + (p9[n] - p9[ls_f]);
                if (l == 0) put_bits(bw, carry_bits, 0, 7);  // 256 = seven zero bits
                carry_bits += 7;
            }
            wsync();
            const uint32_t fixed_bytes = (carry_bits + 7) >> 3, stored_bytes = 5 + n;
            // Adler-32 of the block: A = 1 + sum b, B = n + sum (n - i) b (mod 65521)
            uint64_t sa = 0, sb = 0;
            for (uint32_t i = l; i < n; i += 64) {
                sa += in[i];
                sb += (uint64_t)(n - i) * in[i];
            }
            sa = wave_sum(sa);
            sb = wave_sum(sb);
            const uint32_t A = (uint32_t)((1 + sa) % 65521), B = (uint32_t)((n + sb) % 65521);
            uint32_t p;
            if (fixed_bytes <= stored_bytes) {
                // move the stream from out + 4 down to out + 2 (bytes, ascending: the source is ahead)
                for (uint32_t c0 = 0; c0 < fixed_bytes; c0 += 64) {
                    const uint32_t i = c0 + l;
                    const uint8_t v = i < fixed_bytes ? out[4 + i] : 0;
                    wsync();
                    if (i < fixed_bytes) out[2 + i] = v;
                    wsync();
                }
                p = 2 + fixed_bytes;
            } else {
                for (uint32_t i = l; i < n; i += 64) out[7 + i] = in[i];
                if (l == 0) {
                    out[2] = 1;
                    out[3] = (uint8_t)n; out[4] = (uint8_t)(n >> 8);
                    out[5] = (uint8_t)~n; out[6] = (uint8_t)(~n >> 8);
                }
                p = 7 + n;
            }
            if (l == 0) {
                out[0] = 0x78;
                out[1] = 0x9C;
                out[p] = (uint8_t)(B >> 8); out[p + 1] = (uint8_t)B; out[p + 2] = (uint8_t)(A >> 8); out[p + 3] = (uint8_t)A;
            }
            m = p + 4;
        } else {
            // LZ4 / Snappy: byte elements.  Header: lz4 u32 LE length; snappy varint length.
            uint32_t hdr = 4;
            if (CODEC == SDB_CODEC_SNAPPY) hdr = n < 128 ? 1 : (n < 16384 ? 2 : 3);
            if (l == 0) {
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
            // element sizes: literal header + literals + match element(s)
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
                for (uint32_t j = 0; j < 64 && 64 * ch + j < nseq; j++) {
                    const uint32_t src = (uint32_t)__builtin_amdgcn_readlane((int)lstart, (int)j);
                    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane((int)lit, (int)j);
                    const uint32_t dst = (uint32_t)__builtin_amdgcn_readlane((int)lpos, (int)j);
                    for (uint32_t x = l; x < cnt; x += 64) out[dst + x] = in[src + x];
                }
                carry_out += wave_readlane(oinc, 63);
                carry_pos += wave_readlane(pinc, 63);
            }
            // the final literals (lz4: a last sequence of literals only)
            {
                const uint32_t lit = n - carry_pos;
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
        // d. CRC32 of the compressed bytes (lead-in zeroed: the scratch above may have used it), then the slot
        if (l < 16) ((lu32 *)mm)[l] = 0;
        wsync();
        const uint32_t crc = cz_crc(out, m, (lu8 *)mm + kCzP9Off + 64);
        if (l == 0) {
            out[m] = (uint8_t)(crc >> 24); out[m + 1] = (uint8_t)(crc >> 16); out[m + 2] = (uint8_t)(crc >> 8); out[m + 3] = (uint8_t)crc;
            a.len[k] = m + 4;
        }
        wsync();
        const uint32_t tot = m + 4, n16 = (tot + 15) >> 4;  // slots are 16-byte aligned; out is too
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

static std::once_flag g_cz_once;

uint64_t compress_workspace_bytes(uint64_t nblocks, uint64_t in_bytes) {
    const uint64_t slots = cz_slot(in_bytes, nblocks) + 256;
    const uint64_t nt = (nblocks + 1023) / 1024 + 1;
    return slots + 8 * (nblocks + 2) * 2 + 16 * (nt + 1) + 512;
}

hipError_t launch_compress(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                           uint64_t in_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                           unsigned long long *err, void *ws, hipStream_t st) {
    std::call_once(g_cz_once, [] {
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_LZ4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCzLds);
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_SNAPPY>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCzLds);
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_ZLIB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCzLds);
        (void)hipFuncSetAttribute((const void *)k_cz<SDB_CODEC_ZSTD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCzLds);
        (void)hipGetLastError();
    });
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    CzArgs a{};
    a.codec = codec;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
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
    const uint32_t grid = (uint32_t)((nblocks + kCzWaves - 1) / kCzWaves < 4096 ? (nblocks + kCzWaves - 1) / kCzWaves : 4096);
    switch (codec) {
        case SDB_CODEC_LZ4: hipLaunchKernelGGL(k_cz<SDB_CODEC_LZ4>, dim3(grid), dim3(kCzThreads), kCzLds, st, a); break;
        case SDB_CODEC_SNAPPY: hipLaunchKernelGGL(k_cz<SDB_CODEC_SNAPPY>, dim3(grid), dim3(kCzThreads), kCzLds, st, a); break;
        case SDB_CODEC_ZLIB: hipLaunchKernelGGL(k_cz<SDB_CODEC_ZLIB>, dim3(grid), dim3(kCzThreads), kCzLds, st, a); break;
        default: hipLaunchKernelGGL(k_cz<SDB_CODEC_ZSTD>, dim3(grid), dim3(kCzThreads), kCzLds, st, a); break;
    }
    hipError_t e = launch_excl_scan2(a.len, a.len, nblocks, tx, ty, out_off, scratch, st);
    if (e != hipSuccess) return e;
    const uint32_t pgrid = (uint32_t)((nblocks + 3) / 4 < 4096 ? (nblocks + 3) / 4 : 4096);
    hipLaunchKernelGGL(k_cz_pack, dim3(pgrid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace sdb
