// sdb_codec_ent.hip — device decompression of the entropy-coded block codecs:
//   SDB_CODEC_ZLIB = flate2 1.1.9 read::ZlibDecoder::read_to_end (miniz_oxide 0.8.9): a zlib stream,
//                    RFC 1950 header, RFC 1951 deflate blocks, Adler-32 trailer (format/sst.rs:896-904);
//   SDB_CODEC_ZSTD = zstd 0.13.3 stream::decode_all (libzstd 1.5.7): zstd frames (RFC 8878) and skippable
//                    frames in sequence (format/sst.rs:911-916).
// The crates are not in /root/reference; the formats are restated from their RFCs, with the corner
// semantics of the reference's call sites (header in oracle/sdb_oracle_entropy.c, the CPU restatement
// these kernels are checked against).
//
// Neither format says how long the output is before it is decoded, so both steps decode:
//   E1 plan  one wave per block, lane 0 decodes in count mode (no stores; distances and offsets are
//            still checked against the bytes produced) -> slot = length + 4, or 0 on an error.
//   E2 run   one wave per block: the wave CRC32 of the stored bytes (validate_checksum), lane 0 decodes
//            into the block's slot in HBM (matches read back its own stores), the wave CRC32 of the
//            output, the CRC trailer and out_end.
// (Zlib runs both steps with five decoders per wave, lanes 0-4 each on its own block: k_zl_plan_multi,
// k_zl_run_multi; zstd runs one decoder per wave on all lanes, EntOut::wide and the *_wide table builds.)
// Entropy decoding is serial within a stream, so the parallelism is across blocks (a read_blocks range
// holds hundreds).  Per wave, the LDS holds the code tables: deflate's canonical codes (count + symbols
// by code order), zstd's three FSE sequence tables and the literal Huffman table.  zstd literals are
// decoded straight into the END of the block's own output slot: with o bytes written and lp of the
// block's R literals consumed, the output still to come is at least R - lp, so o <= end - R + lp and
// no store reaches a literal not yet copied.
#include <atomic>
#include <mutex>

#include "sdb_crc.h"
#include "sdb_decode.h"
#include "sdb_device.h"

namespace sdb {

#ifndef SDB_ZS_WFSE
#define SDB_ZS_WFSE 1
#endif
#ifndef SDB_ZS_WHUF
#define SDB_ZS_WHUF 1
#endif
constexpr uint32_t kEntThreads = 768;  // 12 waves per workgroup
constexpr uint64_t kEntMaxOut = 64ull << 20;

struct EntArgs {
    uint32_t codec;
    const uint8_t *blocks;
    const uint64_t *block_off;
    uint64_t nblocks;
    uint64_t *slot;             // plan: per block slot bytes
    uint8_t *out;
    uint64_t out_cap;
    const uint64_t *out_start;  // nblocks + 1
    uint64_t *out_end;
    unsigned long long *err;
    // zlib decode-once (launch_decompress_once): slot i decodes block list[i] (i < *nlist) instead of block
    // i; the optimistic run lists the blocks whose output overflowed their slot instead of failing them,
    // the wide run those with dynamic-Huffman blocks; out_by_block: a list pass writes to out_start[list[i]]
    const uint32_t *list;
    const unsigned long long *nlist;
    uint32_t *ovf_list;
    unsigned long long *ovf_count;
    uint32_t *dyn_list;
    unsigned long long *dyn_count;
    bool out_by_block;
    uint64_t *wres;  // the wide pass's per-block results for k_zl_verify: 2 words per block
};

// ------------------------------------------------------------------------------------------------
// per-wave LDS tables
// ------------------------------------------------------------------------------------------------
struct FseCell {
    uint8_t sym, nb;
    uint16_t base;
};
#ifndef SDB_ZL_FAST_DIST
#define SDB_ZL_FAST_DIST 7
#endif
constexpr int kFastLit = 9, kFastDist = SDB_ZL_FAST_DIST;  // the fast tables' index bits
template <int N>  // N: the alphabet's size (lengths 288, distances 32, code lengths 19)
struct CanonT {
    uint16_t count[16];
    uint16_t sym[N];
};
struct ZTab {  // deflate's code tables
    CanonT<288> lit;
    CanonT<32> dist;
    union {  // the code-length code and the lengths are dead once lit / dist are built from them
        struct {
            CanonT<20> clc;
            uint8_t lens[320];
        };
        struct {
            // 9-bit (lengths) / 7-bit (distances) lookups: sym | len << 12 (len 0: a longer code)
            uint16_t fast_lit[1 << kFastLit], fast_dist[1 << kFastDist];
        };
    };
};
struct EntLds {  // one wave's tables (zlib's alias the zstd ones)
    union {
        ZTab z;
        struct {
            FseCell ll[512], of[256], ml[512], wt[64];  // wt: the Huffman weights' table (accuracy <= 6)
            uint16_t huf[2048];  // sym | nb << 8
            int16_t norm[256];
            uint16_t next[256];
            uint8_t w[256];
            uint32_t llv[36], mlv[53];  // the length codes' baseline | extra bits << 24 (seq_codes_to_lds)
        } s;
    };
};
constexpr uint32_t kEntWaveLds = (sizeof(EntLds) + 15) & ~15u;
constexpr uint32_t kEntLds = 8 * 1024 + (kEntThreads / 64) * kEntWaveLds;
static_assert(kEntLds <= 160 * 1024, "entropy decoder LDS");

// output of one decode: p == nullptr counts only.  wide: every lane of the wave runs this decode with
// the same state (the run kernel), so the byte moves are spread over the lanes: lane l moves 16-byte
// chunks l, l + 64, ... (or bytes l, l + 64, ...) of each copy — the serial decoder's state machine
// stays uniform, only its copies are parallel.  A wave's memory instructions reach memory in program
// order, so a later instruction (any lane) reads what an earlier one stored (as in the one-lane form).
struct EntOut {
    uint8_t *p;
    uint64_t len, cap;
    bool bad;
    bool wide;
    bool adler_defer;     // zlib: leave the Adler-32 check to the caller (adler_want, have_adler)
    bool have_adler;
    uint32_t adler_want;
    SDB_DEV void flush() {}  // (EntOutWC: its pending bytes)
    SDB_DEV uint32_t lane() const { return wide ? (uint32_t)lane_id() : 0u; }
    SDB_DEV uint32_t lanes() const { return wide ? 64u : 1u; }
    SDB_DEV bool put(uint8_t b) {
        if (len >= cap) {
            bad = true;
            return false;
        }
        if (p) p[len] = b;  // (wide: every lane stores the same byte)
        len++;
        return true;
    }
    SDB_DEV bool room(uint64_t n) {
        if (n > cap - len) {
            bad = true;
            return false;
        }
        return true;
    }
    // n bytes from src (not overlapping the output still to be written)
    SDB_DEV bool copy(const uint8_t *src, uint64_t n) {
        if (!room(n)) return false;
        if (p) {
            const uint64_t n16 = n & ~15ull, l = lane(), L = lanes();
            for (uint64_t i = 16 * l; i < n16; i += 16 * L) {
                uint4 w;
                __builtin_memcpy(&w, src + i, 16);
                __builtin_memcpy(p + len + i, &w, 16);
            }
            for (uint64_t i = n16 + l; i < n; i += L) p[len + i] = src[i];
        }
        len += n;
        return true;
    }
    // n copies of byte b (zstd RLE blocks and literals)
    SDB_DEV bool fill(uint8_t b, uint64_t n) {
        if (!room(n)) return false;
        if (p)
            for (uint64_t i = lane(); i < n; i += lanes()) p[len + i] = b;
        len += n;
        return true;
    }
    // n bytes from src >= the write position (zstd's literal stage in the slot), forward.  Chunk i is
    // loaded before it is stored, and no store reaches a source byte a later chunk still reads (src >=
    // dst), so lanes may move consecutive chunks at once for any src - dst >= 16; a closer source goes
    // bytewise in order on one lane.
    SDB_DEV bool copy_fwd(const uint8_t *src, uint64_t n) {
        if (!room(n)) return false;
        uint8_t *dst = p + len;
        uint64_t i = 0;
        if (src - dst >= 16) {
            const uint64_t n16 = n & ~15ull, l = lane(), L = lanes();
            for (uint64_t j = 16 * l; j < n16; j += 16 * L) {
                uint4 w;
                __builtin_memcpy(&w, src + j, 16);
                __builtin_memcpy(dst + j, &w, 16);
            }
            for (uint64_t j = n16 + l; j < n; j += L) dst[j] = src[j];
            i = n;
        }
        if (src != dst)
            for (; i < n; i++) dst[i] = src[i];
        len += n;
        return true;
    }
    // a match of n bytes at distance d: byte i comes from len - d + (i mod d), always below len (a
    // byte written before this call), so every byte can move at once; one lane: 16 at a time when d >= 16
    SDB_DEV bool match(uint64_t d, uint64_t n) {
        if (!room(n)) return false;
        if (p) {
            if (wide) {
                const uint8_t *src = p + len - d;  // d <= the output so far (the callers check)
                const uint32_t d32 = d < 0x80000000ull ? (uint32_t)d : 0x80000000u;
                uint64_t i = lane_id(), r = d > 64 ? i : (uint32_t)i % d32;
                const uint64_t step = d > 64 ? 64 : 64u % d32;
                for (; i < n; i += 64) {
                    p[len + i] = src[r];
                    r += step;
                    r = r >= d ? r - d : r;
                }
            } else {
                uint64_t i = 0;
                if (d >= 16)
                    for (; i + 16 <= n; i += 16) {
                        uint4 w;
                        __builtin_memcpy(&w, p + len - d + i, 16);
                        __builtin_memcpy(p + len + i, &w, 16);
                    }
                for (; i < n; i++) p[len + i] = p[len + i - d];
            }
        }
        len += n;
        return true;
    }
};

// One-lane decoder output with the literals gathered into 8-byte stores (k_zl_run_multi): the last pn
// bytes of the output wait in pend; every call that reads or writes p otherwise flushes them first.
struct EntOutWC : EntOut {
    uint32_t pn;
    uint64_t pend;
    SDB_DEV bool put(uint8_t b) {
        if (len >= cap) {
            bad = true;
            return false;
        }
        pend |= (uint64_t)b << (8 * pn);
        len++;
        if (++pn == 8) {
            __builtin_memcpy(p + len - 8, &pend, 8);
            pend = 0;
            pn = 0;
        }
        return true;
    }
    // one 8-byte store when it stays inside the slot and its CRC trailer (cap + 4; the bytes past len
    // are written again, in order, before anything reads them), else bytewise
    SDB_DEV void flush() {
        if (!pn) return;
        if (len - pn + 8 <= cap + 4) {
            __builtin_memcpy(p + len - pn, &pend, 8);
        } else {
            for (uint32_t i = 0; i < pn; i++) p[len - pn + i] = (uint8_t)(pend >> (8 * i));
        }
        pend = 0;
        pn = 0;
    }
    SDB_DEV bool copy(const uint8_t *src, uint64_t n) {
        flush();
        return EntOut::copy(src, n);
    }
    SDB_DEV bool match(uint64_t d, uint64_t n) {
        flush();
        return EntOut::match(d, n);
    }
};

// EntOutWC for a wave of decoders (the wide zlib pass): each lane also keeps the last 256 bytes of its output
// in an LDS column (byte i at ring[(i & 255) * 64]), so a match within 256 bytes copies from LDS instead of
// loading the lane's own fresh stores back from memory (with 64 lanes decoding, some lane's match would
// otherwise wait on memory at nearly every symbol).
struct EntOutRing : EntOutWC {
    lu8 *ring;
    SDB_DEV bool put(uint8_t b) {
        if (len >= cap) {
            bad = true;
            return false;
        }
        ring[(uint32_t)(len & 255) * 64] = b;
        return EntOutWC::put(b);
    }
    // c <= 8 bytes (the low bytes of w, the rest zero) at once: ring writes, then one merge with the
    // pending bytes (an 8-byte store when they reach 8).  The caller has checked room(c).
    SDB_DEV void put_n(uint64_t w, uint32_t c) {
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
            if (j < c) ring[(uint32_t)((len + j) & 255) * 64] = (uint8_t)(w >> (8 * j));
        if (pn + c < 8) {
            pend |= w << (8 * pn);
            pn += c;
        } else {
            const uint64_t out = pend | (w << (8 * pn));
            __builtin_memcpy(p + len - pn, &out, 8);
            const uint32_t rem = pn + c - 8;
            pend = rem ? w >> (8 * (8 - pn)) : 0;
            pn = rem;
        }
        len += c;
    }
    // the next c <= 8 bytes of a match at distance d (the step machine of zlib_decode_wide)
    SDB_DEV bool copy_step(uint64_t d, uint32_t c) {
        if (!room(c)) return false;
        if (d > 256) {  // older bytes: from the lane's own stores, one at a time (rare)
            flush();
            for (uint32_t i = 0; i < c; i++) put(p[len - d]);
            return true;
        }
        uint64_t w = 0;
        const uint32_t dd = (uint32_t)d;
        if (dd >= 8) {
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) w |= (uint64_t)ring[(uint32_t)((len - dd + j) & 255) * 64] << (8 * j);
        } else {  // an overlapping match: byte j repeats byte j mod d of the last d
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) w |= (uint64_t)ring[(uint32_t)((len - dd + j % dd) & 255) * 64] << (8 * j);
        }
        if (c < 8) w &= (1ull << (8 * c)) - 1;
        put_n(w, c);
        return true;
    }
    SDB_DEV bool match(uint64_t d, uint64_t n) {
        if (!room(n)) return false;
        if (d <= 256) {
            uint64_t i = 0;
            if (d >= 8)  // eight reads in flight, then eight puts (no byte of a batch is one it reads)
                for (; i + 8 <= n; i += 8) {
                    uint8_t v[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) v[j] = ring[(uint32_t)((len - d + j) & 255) * 64];
#pragma unroll
                    for (int j = 0; j < 8; j++) put(v[j]);
                }
            for (; i < n; i++) put(ring[(uint32_t)((len - d) & 255) * 64]);
            return true;
        }
        flush();  // older bytes: from the lane's own stores, one at a time (rare: distances over 256)
        for (uint64_t i = 0; i < n; i++) put(p[len - d]);
        return true;
    }
};

// ------------------------------------------------------------------------------------------------
// zlib / deflate
// ------------------------------------------------------------------------------------------------
struct LsbBits {  // the 4 bytes after the stream (its block's CRC32 trailer) are readable
    const uint8_t *p;
    uint64_t n, pos;
    uint64_t buf;
    int cnt;
    uint64_t nw;   // the 8 bytes from pos, loaded one refill ahead (n >= 4): raw, then >> nsh bits at use
    uint32_t nsh;
    // the load for 8 bytes from `at` (<= n): it stays inside the stream and its trailer, at most 3 bytes
    // back from the end (shifted out at use, so the load's wait comes at the next refill)
    SDB_DEV void load_at(uint64_t at) {
        const uint64_t q = at + 4 <= n ? at : n - 4;
        __builtin_memcpy(&nw, p + q, 8);
        nsh = 8 * (uint32_t)(at - q);
    }
    SDB_DEV void start() {
        nw = 0;
        nsh = 0;
        if (n >= 4) load_at(pos);
    }
    SDB_DEV void refill() {  // to >= 56 bits (fewer at the stream's end)
        if (cnt >= 56 || pos >= n) return;
        if (n < 4) {  // (a stream too short to hold a header)
            while (cnt <= 56 && pos < n) {
                buf |= (uint64_t)p[pos++] << cnt;
                cnt += 8;
            }
            return;
        }
        // the bytes past the whole ones taken (or past the stream) land above cnt, where a later refill ORs
        // the same bytes at the same bit positions, and nothing reads them as input
        buf |= (nw >> nsh) << cnt;
        uint64_t take = (63 - (uint32_t)cnt) >> 3;
        if (take > n - pos) take = n - pos;
        pos += take;
        cnt += 8 * (int)take;
        load_at(pos);  // in flight while this refill's bits are decoded
    }
    SDB_DEV bool get(int k, uint32_t &v) {  // k <= 16; false when the input ends first
        if (cnt < k) refill();
        if (cnt < k) return false;
        v = (uint32_t)(buf & ((1ull << k) - 1));
        buf >>= k;
        cnt -= k;
        return true;
    }
    SDB_DEV void align() {
        buf >>= cnt & 7;
        cnt -= cnt & 7;
    }
};

template <int N>
SDB_DEV int canon_build(CanonT<N> &h, const uint8_t *len, int n) {
    uint16_t offs[16];
    for (int l = 0; l < 16; l++) h.count[l] = 0;
    for (int s = 0; s < n; s++) h.count[len[s]]++;
    const int used = n - h.count[0];
    int left = 1;
    for (int l = 1; l < 16; l++) {
        left <<= 1;
        left -= h.count[l];
        if (left < 0) return used > 1 ? -1 : 0;
    }
    if (left > 0 && used > 1) return -1;
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + h.count[l];
    for (int s = 0; s < n; s++)
        if (len[s]) h.sym[offs[len[s]]++] = (uint16_t)s;
    return 0;
}

// the K-bit fast table of a usable code: every code of <= K bits, bit-reversed (deflate sends a code's
// bits most significant first into an LSB-first stream), replicated over the bits that follow it
template <int K, int N>
SDB_DEV void canon_fast(const CanonT<N> &h, uint16_t *fast) {
    for (int i = 0; i < (1 << K); i++) fast[i] = 0;
    int code = 0, index = 0;
    for (int l = 1; l <= K; l++) {
        for (int c = 0; c < h.count[l]; c++, code++, index++) {
            const int r = (int)(__builtin_bitreverse32((uint32_t)code) >> (32 - l));
            const uint16_t e = (uint16_t)(h.sym[index] | l << 12);
            for (int j = r; j < (1 << K); j += 1 << l) fast[j] = e;
        }
        code <<= 1;
    }
}

// -1 input ended, -2 invalid code: the code's bits MSB first from the buffer (one refill, no per-bit input)
template <int N>
SDB_DEV int canon_decode(LsbBits &s, const CanonT<N> &h) {
    if (s.cnt < 15) s.refill();
    int code = 0, first = 0, index = 0;
#pragma unroll 1
    for (int l = 1; l < 16; l++) {
        if (l > s.cnt) return -1;
        code |= (int)((s.buf >> (l - 1)) & 1);
        const int c = h.count[l];
        if (code - first < c) {
            s.buf >>= l;
            s.cnt -= l;
            return h.sym[index + code - first];
        }
        index += c;
        first += c;
        first <<= 1;
        code <<= 1;
    }
    return -2;
}

// deflate's length symbols 257 + i and distance symbols ds: base and extra bits (RFC 1951 3.2.5)
SDB_DEV uint32_t len_extra(int i) { return i < 8 || i == 28 ? 0u : (uint32_t)(i - 4) >> 2; }
SDB_DEV uint32_t len_base(int i) {
    return i < 8 ? 3u + i : i == 28 ? 258u : ((4u + (i & 3)) << ((uint32_t)(i - 4) >> 2)) + 3u;
}
SDB_DEV uint32_t dist_extra(int ds) { return ds < 4 ? 0u : (uint32_t)(ds >> 1) - 1u; }
SDB_DEV uint32_t dist_base(int ds) { return ds < 4 ? 1u + ds : ((2u + (ds & 1)) << ((ds >> 1) - 1)) + 1u; }
__constant__ uint8_t c_cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { kZOk = 0, kZTrunc = 1, kZErr = -1, kZDyn = 2 };

// deflate's fixed code (RFC 1951 3.2.6) in t, written by the whole workgroup (tid of nt) in closed form: the
// canonical codes of the fixed lengths are 7-bit 0..23 (symbols 256..279), 8-bit 48..191 (0..143) and
// 192..199 (280..287), 9-bit 400..511 (144..255), distances 5-bit 0..31; a fast-table index read LSB first
// is the code's bits reversed
SDB_DEV void zl_fixed_tables(ZTab &t, uint32_t tid, uint32_t nt) {
    for (uint32_t i = tid; i < (1u << kFastLit); i += nt) {
        const uint32_t r9 = __builtin_bitreverse32(i) >> 23, p8 = r9 >> 1;
        uint32_t e;
        if (r9 < 96) e = (256 + (r9 >> 2)) | 7u << 12;
        else if (p8 < 192) e = (p8 - 48) | 8u << 12;
        else if (p8 < 200) e = (280 + p8 - 192) | 8u << 12;
        else e = (144 + r9 - 400) | 9u << 12;
        t.fast_lit[i] = (uint16_t)e;
    }
    for (uint32_t i = tid; i < (1u << kFastDist); i += nt)
        t.fast_dist[i] = (uint16_t)((__builtin_bitreverse32(i & 31) >> 27) | 5u << 12);
    for (uint32_t j = tid; j < 288; j += nt)  // by length, then symbol
        t.lit.sym[j] = (uint16_t)(j < 24 ? 256 + j : j < 168 ? j - 24 : j < 176 ? 280 + j - 168 : 144 + j - 176);
    for (uint32_t j = tid; j < 32; j += nt) t.dist.sym[j] = (uint16_t)j;
    for (uint32_t l = tid; l < 16; l += nt) {
        t.lit.count[l] = (uint16_t)(l == 7 ? 24 : l == 8 ? 152 : l == 9 ? 112 : 0);
        t.dist.count[l] = (uint16_t)(l == 5 ? 32 : 0);
    }
}

#ifndef SDB_ZL_UNIFORM_REFILL
#define SDB_ZL_UNIFORM_REFILL 1
#endif
#ifndef SDB_ZL_REFILL_AT
#define SDB_ZL_REFILL_AT 9  // (bits under which a wave refills: a literal / length code needs at most 9 here)
#endif
// SHARED: t holds the fixed code's tables (zl_fixed_tables), read-only and shared by the decoders of a
// workgroup; a dynamic-Huffman block returns kZDyn (its decoder has no tables of its own)
template <bool SHARED = false, class Out>
SDB_DEV int inflate_raw(LsbBits &s, Out &o, ZTab &t) {
    uint32_t last = 0;
    uint8_t *lens = t.lens;
    do {
        uint32_t type;
        if (!s.get(1, last) || !s.get(2, type)) return kZTrunc;
        if (type == 0) {
            s.align();
            uint32_t ln, nl;
            if (!s.get(16, ln) || !s.get(16, nl)) return kZTrunc;
            if ((ln ^ 0xFFFF) != nl) return kZErr;
            // the whole bytes left in the bit buffer, then straight from the stream 32 bytes per step (four
            // loads in flight instead of a refill every 7 bytes); the bit reader restarts after them
            uint32_t i = 0;
            for (; i < ln && s.cnt >= 8; i++) {
                if (!o.put((uint8_t)s.buf)) return kZErr;
                s.buf >>= 8;
                s.cnt -= 8;
            }
            const uint64_t avail = s.n - s.pos < (uint64_t)(ln - i) ? s.n - s.pos : (uint64_t)(ln - i);
            const uint8_t *src = s.p + s.pos;
            uint64_t c = 0;
            for (; c + 32 <= avail; c += 32) {
                uint64_t w[4];
                __builtin_memcpy(w, src + c, 32);
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int j = 0; j < 8; j++)
                        if (!o.put((uint8_t)(w[q] >> (8 * j)))) return kZErr;
            }
            for (; c < avail; c++)
                if (!o.put(src[c])) return kZErr;
            s.pos += avail;
            s.buf = s.cnt ? s.buf & ((1ull << s.cnt) - 1) : 0;  // (cnt < 8 here: stale bits above it cleared)
            if (s.n >= 4) s.load_at(s.pos);
            if (i + avail < ln) return kZTrunc;
            continue;
        }
        if (type == 3) return kZErr;
        if constexpr (SHARED) {
            if (type == 2) return kZDyn;
        }
        int nlen, ndist;
        if (SHARED) {
            // the fixed code's tables are already in t
        } else if (type == 1) {
            for (int i = 0; i < 288; i++) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
            for (int i = 0; i < 32; i++) lens[288 + i] = 5;
            nlen = 288;
            ndist = 32;
        } else {
            uint32_t hlit, hdist, hclen;
            if (!s.get(5, hlit) || !s.get(5, hdist) || !s.get(4, hclen)) return kZTrunc;
            nlen = (int)hlit + 257;
            ndist = (int)hdist + 1;
            if (nlen > 286 || ndist > 30) return kZErr;
            uint8_t cl[19];
            for (int i = 0; i < 19; i++) cl[i] = 0;
            for (uint32_t i = 0; i < hclen + 4; i++) {
                uint32_t v;
                if (!s.get(3, v)) return kZTrunc;
                cl[c_cl_order[i]] = (uint8_t)v;
            }
            if (canon_build(t.clc, cl, 19)) return kZErr;
            int i = 0;
            while (i < nlen + ndist) {
                const int sym = canon_decode(s, t.clc);
                if (sym == -1) return kZTrunc;
                if (sym < 0) return kZErr;
                if (sym < 16) {
                    lens[i++] = (uint8_t)sym;
                    continue;
                }
                uint32_t rep, v;
                uint8_t val = 0;
                if (sym == 16) {
                    if (i == 0) return kZErr;
                    val = lens[i - 1];
                    if (!s.get(2, v)) return kZTrunc;
                    rep = 3 + v;
                } else if (sym == 17) {
                    if (!s.get(3, v)) return kZTrunc;
                    rep = 3 + v;
                } else {
                    if (!s.get(7, v)) return kZTrunc;
                    rep = 11 + v;
                }
                if (i + (int)rep > nlen + ndist) return kZErr;
                while (rep--) lens[i++] = val;
            }
            if (lens[256] == 0) return kZErr;
            for (int q = ndist - 1; q >= 0; q--) lens[288 + q] = lens[nlen + q];
        }
        if (!SHARED) {
            if (canon_build(t.lit, lens, nlen) || canon_build(t.dist, lens + 288, ndist)) return kZErr;
            canon_fast<kFastLit>(t.lit, t.fast_lit);
            canon_fast<kFastDist>(t.dist, t.fast_dist);
        }
        // a symbol through the fast table (mask: its size - 1) when its code is short enough and the bits
        // are there
        auto fast_decode = [&](const uint16_t *fast, uint32_t mask, const auto &h) -> int {
            if constexpr (SHARED || SDB_ZL_UNIFORM_REFILL) {
                // a wave of decoders: when any lane runs low, every lane here refills and stores its pending
                // output bytes, so the loads and stores a refill's wait covers were issued a refill ago
                // (lane by lane, some lane's fresh load or store would be waited on at every symbol)
                if (__ballot(s.cnt < SDB_ZL_REFILL_AT)) {
                    s.refill();
                    o.flush();
                }
            } else if (s.cnt < 9) {
                s.refill();
            }
            const uint16_t e = fast[s.buf & mask];
            const int L = e >> 12;
            if (L && L <= s.cnt) {
                s.buf >>= L;
                s.cnt -= L;
                return e & 0xFFF;
            }
            return canon_decode(s, h);
        };
        for (;;) {
            int sym = fast_decode(t.fast_lit, (1u << kFastLit) - 1, t.lit);
            if (sym == -1) return kZTrunc;
            if (sym < 0) return kZErr;
            if (sym < 256) {
                if (!o.put((uint8_t)sym)) return kZErr;
                continue;
            }
            if (sym == 256) break;
            sym -= 257;
            if (sym >= 29) return kZErr;
            uint32_t v;
            if (!s.get((int)len_extra(sym), v)) return kZTrunc;
            const uint32_t len = len_base(sym) + v;
            const int ds = fast_decode(t.fast_dist, (1u << kFastDist) - 1, t.dist);
            if (ds == -1) return kZTrunc;
            if (ds < 0 || ds >= 30) return kZErr;
            if (!s.get((int)dist_extra(ds), v)) return kZTrunc;
            const uint32_t d = dist_base(ds) + v;
            if (d > o.len) return kZErr;
            if (!o.match(d, len)) return kZErr;
        }
    } while (!last);
    return kZOk;
}

// 0 or -1; Adler-32 checked when the bytes are kept
// 0, -1, or (SHARED) 1: a dynamic-Huffman block, left to a decoder with its own tables
template <bool SHARED = false, class Out>
SDB_DEV int zlib_decode(const uint8_t *in, uint64_t n, Out &o, ZTab &t) {
    if (n < 2) return 0;
    const uint32_t cmf = in[0], flg = in[1];
    if ((cmf & 0x0F) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return -1;
    LsbBits s{in, n, 2, 0, 0, 0, 0};
    s.start();
    const int r = inflate_raw<SHARED>(s, o, t);
    if (r == kZDyn) return 1;
    if (r == kZErr) return -1;
    if (r == kZTrunc) return 0;
    s.align();
    uint32_t a = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t b;
        if (!s.get(8, b)) return 0;
        a = a << 8 | b;
    }
    if (o.p && o.adler_defer) {  // the caller checks it (a whole wave, after the decode)
        o.have_adler = true;
        o.adler_want = a;
    } else if (o.p && o.wide) {
        // Adler-32 over n bytes as sums: A = 1 + sum b_i, B = n + sum (n - i) b_i (mod 65521), lane l
        // taking bytes l, l + 64, ... (coalesced); (n - i) b_i < 2^34 and a lane adds at most 2^20 of
        // them per 64 MiB, so the u64 sums never wrap
        const uint64_t n = o.len;
        uint64_t sa = 0, sb = 0;
        for (uint64_t i = (uint64_t)lane_id(); i < n; i += 64) {
            const uint64_t b = o.p[i];
            sa += b;
            sb += (n - i) * b;
        }
        sa = wave_sum(sa);
        sb = wave_sum(sb);
        const uint32_t x = (uint32_t)((1 + sa) % 65521u), y = (uint32_t)((n % 65521u + sb % 65521u) % 65521u);
        if ((y << 16 | x) != a) return -1;
    } else if (o.p) {
        uint32_t x = 1, y = 0;
        for (uint64_t i = 0; i < o.len; i++) {
            x += o.p[i];
            if (x >= 65521u) x -= 65521u;
            y += x;
            if (y >= 65521u) y -= 65521u;
        }
        if ((y << 16 | x) != a) return -1;
    }
    return 0;
}

// The wide pass's inflate (k_zl_wide: 64 decoders per wave on the fixed code's shared tables) as a step
// machine: every iteration each lane does one short step — a block header, one symbol, or up to 8 bytes
// of a pending match — so lanes that meet a match do not hold the others through its whole copy (the
// divergent literal and match paths of inflate_raw ran one after the other for all 64 lanes).  Refills
// and the pending output stores happen at wave-uniform points (any lane under 32 bits: every step needs
// at most 9 + 5 + 5 + 13).  Returns what zlib_decode<true> returns: 0, -1, or 1 for a dynamic block.
SDB_DEV int zlib_decode_wide(const uint8_t *in, uint64_t n, EntOutRing &o, const ZTab &t) {
    if (n < 2) return 0;
    const uint32_t cmf = in[0], flg = in[1];
    if ((cmf & 0x0F) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return -1;
    LsbBits s{in, n, 2, 0, 0, 0, 0};
    s.start();
    int r = kZOk;
    uint32_t last = 0, mlen = 0, mdist = 0;
    bool hdr = true, fin = false;
    while (!fin) {
        if (__ballot(s.cnt < 32)) {
            s.refill();
            o.flush();
        }
        if (mlen) {  // a pending match: up to 8 bytes this step
            const uint32_t c = mlen < 8 ? mlen : 8;
            if (!o.copy_step(mdist, c)) {
                r = kZErr;
                fin = true;
            }
            mlen -= c;
            continue;
        }
        if (hdr) {  // the next deflate block's header, or the end of the last one
            uint32_t type = 0;
            if (last) {
                fin = true;
            } else if (!s.get(1, last) || !s.get(2, type)) {
                r = kZTrunc;
                fin = true;
            } else if (type == 2 || type == 3) {
                r = type == 2 ? kZDyn : kZErr;
                fin = true;
            } else if (type == 1) {
                hdr = false;
            } else {  // stored: the whole block in one step (bytes left in the buffer, then 32 per load)
                s.align();
                uint32_t ln, nl;
                if (!s.get(16, ln) || !s.get(16, nl)) {
                    r = kZTrunc;
                    fin = true;
                    continue;
                }
                if ((ln ^ 0xFFFF) != nl) {
                    r = kZErr;
                    fin = true;
                    continue;
                }
                uint32_t i = 0;
                bool ok = true;
                for (; i < ln && s.cnt >= 8 && ok; i++) {
                    ok = o.put((uint8_t)s.buf);
                    s.buf >>= 8;
                    s.cnt -= 8;
                }
                const uint64_t avail = s.n - s.pos < (uint64_t)(ln - i) ? s.n - s.pos : (uint64_t)(ln - i);
                const uint8_t *src = s.p + s.pos;
                for (uint64_t c = 0; c < avail && ok; c += 8) {
                    const uint32_t k = avail - c < 8 ? (uint32_t)(avail - c) : 8;
                    uint64_t w = 0;
                    if (k == 8) __builtin_memcpy(&w, src + c, 8);
                    else
                        for (uint32_t j = 0; j < k; j++) w |= (uint64_t)src[c + j] << (8 * j);
                    ok = o.room(k);
                    if (ok) o.put_n(w, k);
                }
                s.pos += avail;
                s.buf = s.cnt ? s.buf & ((1ull << s.cnt) - 1) : 0;
                if (s.n >= 4) s.load_at(s.pos);
                if (!ok) {
                    r = kZErr;
                    fin = true;
                } else if (i + avail < ln) {
                    r = kZTrunc;
                    fin = true;
                }
            }
            continue;
        }
        // one symbol of a fixed-code block (every fixed literal / length code is in the 9-bit table)
        int sym;
        {
            const uint16_t e = t.fast_lit[s.buf & ((1u << kFastLit) - 1)];
            const int L = e >> 12;
            if (L && L <= s.cnt) {
                s.buf >>= L;
                s.cnt -= L;
                sym = e & 0xFFF;
            } else {
                sym = canon_decode(s, t.lit);
            }
        }
        if (sym < 0) {
            r = sym == -1 ? kZTrunc : kZErr;
            fin = true;
        } else if (sym < 256) {
            if (!o.put((uint8_t)sym)) {
                r = kZErr;
                fin = true;
            }
        } else if (sym == 256) {
            hdr = true;
        } else if (sym - 257 >= 29) {
            r = kZErr;
            fin = true;
        } else {
            uint32_t v;
            const int ls = sym - 257;
            if (!s.get((int)len_extra(ls), v)) {
                r = kZTrunc;
                fin = true;
                continue;
            }
            const uint32_t len = len_base(ls) + v;
            int ds;
            {
                const uint16_t e = t.fast_dist[s.buf & ((1u << kFastDist) - 1)];
                const int L = e >> 12;
                if (L && L <= s.cnt) {
                    s.buf >>= L;
                    s.cnt -= L;
                    ds = e & 0xFFF;
                } else {
                    ds = canon_decode(s, t.dist);
                }
            }
            if (ds == -1 || (ds >= 0 && ds < 30 && !s.get((int)dist_extra(ds), v))) {
                r = kZTrunc;
                fin = true;
            } else if (ds < 0 || ds >= 30 || dist_base(ds) + v > o.len) {
                r = kZErr;
                fin = true;
            } else {
                mlen = len;
                mdist = dist_base(ds) + v;
            }
        }
    }
    if (r == kZDyn) return 1;
    if (r == kZErr) return -1;
    if (r == kZTrunc) return 0;
    s.align();
    uint32_t a = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t b;
        if (!s.get(8, b)) return 0;
        a = a << 8 | b;
    }
    o.have_adler = true;  // (k_zl_verify checks it)
    o.adler_want = a;
    return 0;
}

// ------------------------------------------------------------------------------------------------
// zstd
// ------------------------------------------------------------------------------------------------
SDB_DEV int hb32(uint32_t v) { return 31 - __builtin_clz(v); }
SDB_DEV uint32_t rd32b(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

// backward bitstream, most significant bit first from the last byte's marker
struct RevBits {
    const uint8_t *p;
    int64_t n, pos, wb;
    uint64_t win;
    SDB_DEV void load(int64_t w0) {
        wb = w0;
        uint64_t v = 0;
        const int64_t b0 = w0 >> 3;
        if (b0 + 8 <= n) {
            __builtin_memcpy(&v, p + b0, 8);  // one unaligned 8-byte load
        } else {
            for (int i = 0; i < 8; i++)
                if (b0 + i < n) v |= (uint64_t)p[b0 + i] << (8 * i);
        }
        win = v;
    }
    SDB_DEV bool init(const uint8_t *q, int64_t len) {
        p = q;
        n = len;
        if (len == 0 || q[len - 1] == 0) return false;
        pos = (len - 1) * 8 + hb32(q[len - 1]);
        int64_t w = pos - 64 + 7;
        load(w > 0 ? (w >> 3) << 3 : 0);
        return true;
    }
    SDB_DEV uint32_t peek(int k) {  // k <= 32; bits below 0 read as 0
        if (k == 0) return 0;
        const int64_t lo = pos - k;
        if (lo < wb && wb > 0) {
            int64_t w = pos - 64 + 7;
            load(w > 0 ? (w >> 3) << 3 : 0);
        }
        if (lo >= 0) return (uint32_t)((win >> (lo - wb)) & ((1ull << k) - 1));
        if (pos <= 0) return 0;
        const uint32_t have = (uint32_t)((win >> (0 - wb)) & ((1ull << pos) - 1));  // wb == 0 here
        return have << (uint32_t)(-lo);
    }
    SDB_DEV uint32_t get(int k) {
        const uint32_t v = peek(k);
        pos -= k;
        return v;
    }
};

// an FSE cell {sym, nb, base} as one dword: sym | nb << 8 | base << 16
SDB_DEV uint32_t fse_cell(const FseCell *t, uint32_t st) {
    uint32_t v;
    __builtin_memcpy(&v, t + st, 4);
    return v;
}

SDB_DEV int fse_build(FseCell *t, int16_t *norm, uint16_t *next, int nsym, int al) {
    const int size = 1 << al;
    int high = size - 1;
    for (int s = 0; s < nsym; s++) {
        if (norm[s] == -1) {
            t[high--].sym = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)norm[s];
        }
    }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int pos = 0;
    for (int s = 0; s < nsym; s++)
        for (int i = 0; i < norm[s]; i++) {
            t[pos].sym = (uint8_t)s;
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    if (pos != 0) return -1;
    for (int u = 0; u < size; u++) {
        const int s = t[u].sym;
        const uint32_t x = next[s]++;
        const int nb = al - hb32(x);
        t[u].nb = (uint8_t)nb;
        t[u].base = (uint16_t)((x << nb) - (uint32_t)size);
    }
    return 0;
}

// The same table built by the whole wave (every lane calls it with the same arguments), for tables of
// <= 64 cells and <= 64 symbols (all of zstd's predefined tables; accuracy log 6 or less): lane s holds
// symbol s's count, lane k the spread's k-th step.  Step k lands on cell (k * step) & mask; the steps
// that land below the low-probability cells take the positive-count cells in symbol order (ballot rank
// of the valid steps), and a cell's state counter is its symbol's count plus the cell's rank among that
// symbol's cells in cell order (a ballot per symbol).  Other tables: the serial build.
__device__ __attribute__((noinline)) int fse_build_wide(FseCell *t, int16_t *norm, uint16_t *next, int nsym, int al) {
    const int size = 1 << al;
    if (!SDB_ZS_WFSE || size > 64 || nsym > 64) return fse_build(t, norm, next, nsym, al);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // norm, as every lane stored it
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t lt = (1ull << l) - 1;
    const int ns = (int)l < nsym ? norm[l] : 0;
    const uint32_t npos = ns > 0 ? (uint32_t)ns : 0u;
    const uint64_t mlow = __ballot(ns == -1);
    const int high = size - 1 - __popcll(mlow);
    const uint32_t incl = wave_incl_scan(npos), total = wave_readlane(incl, 63), cum = incl - npos;
    if ((int)total != high + 1) return fse_build(t, norm, next, nsym, al);
    uint16_t *symc = next;  // scratch: the symbol of the c-th positive cell (norm stays in registers)
    for (uint32_t i = 0; i < npos; i++) symc[cum + i] = (uint16_t)l;
    if (ns == -1) t[size - 1 - __popcll(mlow & lt)].sym = (uint8_t)l;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    const int pk = ((int)l * step) & mask;
    const bool valid = (int)l < size && pk <= high;
    const uint32_t c = (uint32_t)__popcll(__ballot(valid) & lt);
    if (valid) t[pk].sym = (uint8_t)symc[c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool cell = (int)l < size;
    const uint32_t sym = cell ? t[l].sym : 0xFFu;
    uint32_t rank = 0;
    for (int q = 0; q < nsym; q++) {
        const uint64_t m = __ballot(sym == (uint32_t)q);
        if (sym == (uint32_t)q) rank = (uint32_t)__popcll(m & lt);
    }
    const uint32_t nx = (uint32_t)__shfl(ns == -1 ? 1 : ns, cell ? (int)sym : 0, 64);
    if (cell) {
        const uint32_t x = nx + rank;
        const int nb = al - hb32(x);
        t[l].nb = (uint8_t)nb;
        t[l].base = (uint16_t)((x << nb) - (uint32_t)size);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return 0;
}

// FSE table description (forward, LSB-first) -> norm; bytes used or -1
SDB_DEV int fse_read_ncount(const uint8_t *in, uint64_t n, int16_t *norm, int *nsym, int max_sym, int max_al, int *al_out) {
    if (n < 1) return -1;
    // bits [bitpos, bitpos + k) LSB-first, those past the end reading as 0, from a 64-bit window (one
    // unaligned 8-byte load per <= 57 bits)
    uint64_t bitpos = 0, wbase = 0, win = 0;
    auto load = [&]() {
        const uint64_t b0 = bitpos >> 3;
        wbase = b0 << 3;
        uint64_t v = 0;
        if (b0 + 8 <= n) {
            __builtin_memcpy(&v, in + b0, 8);
        } else {
            for (uint64_t i = 0; i < 8; i++)
                if (b0 + i < n) v |= (uint64_t)in[b0 + i] << (8 * i);
        }
        win = v;
    };
    load();
    auto bits = [&](int k) -> uint32_t {  // k <= 16
        if (bitpos + (uint64_t)k > wbase + 64) load();
        return (uint32_t)((win >> (bitpos - wbase)) & ((1u << k) - 1));
    };
    const int al = (int)bits(4) + 5;
    bitpos += 4;
    if (al > max_al) return -1;
    int remaining = (1 << al) + 1, threshold = 1 << al, nbits = al + 1, s = 0;
    while (remaining > 1 && s <= max_sym) {
        const int mx = (2 * threshold - 1) - remaining;
        int v;
        const uint32_t low = bits(nbits - 1);
        if ((int)low < mx) {
            v = (int)low;
            bitpos += nbits - 1;
        } else {
            v = (int)bits(nbits);
            if (v >= threshold) v -= mx;
            bitpos += nbits;
        }
        const int proba = v - 1;
        remaining -= proba < 0 ? -proba : proba;
        norm[s++] = (int16_t)proba;
        if (proba == 0) {
            for (;;) {
                const int r = (int)bits(2);
                bitpos += 2;
                for (int i = 0; i < r && s <= max_sym; i++) norm[s++] = 0;
                if (r != 3) break;
            }
        }
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
    }
    if (remaining != 1 || s > max_sym + 1) return -1;
    if ((bitpos + 7) / 8 > n) return -1;
    *nsym = s;
    *al_out = al;
    return (int)((bitpos + 7) / 8);
}

SDB_DEV int huf_from_weights(EntLds &t, int nw, int *maxbits_out) {
    uint8_t *w = t.s.w;
    uint32_t total = 0;
    for (int i = 0; i < nw; i++) {
        if (w[i] > 11) return -1;
        if (w[i]) total += 1u << (w[i] - 1);
    }
    if (total == 0) return -1;
    const int maxbits = hb32(total) + 1;
    if (maxbits > 11) return -1;
    const uint32_t rest = (1u << maxbits) - total;
    if (rest & (rest - 1)) return -1;
    w[nw] = (uint8_t)(hb32(rest) + 1);
    const int ns = nw + 1;
    uint32_t p = 0;
    for (int wv = 1; wv <= maxbits; wv++)
        for (int s = 0; s < ns; s++) {
            if (w[s] != wv) continue;
            const uint16_t e = (uint16_t)(s | (maxbits + 1 - wv) << 8);
            for (uint32_t i = 0; i < (1u << (wv - 1)); i++) t.s.huf[p++] = e;
        }
    *maxbits_out = maxbits;
    return 0;
}

// The same table built by the whole wave (every lane calls it with the same arguments): symbol s of
// weight v owns the run of 2^(v-1) cells starting at the cells of every lighter symbol and of every
// lower symbol of the same weight (ballot ranks per weight), each run's first cell takes its entry and
// the cells between are filled forward from the last entry before them (a wave max-scan over lanes'
// 32-cell segments).  The serial fill walks weight x symbol: ≈ 2,800 steps per table.
__device__ __attribute__((noinline)) int huf_from_weights_wide(EntLds &t, int nw, int *maxbits_out) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the weights every lane stored
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint8_t *w = t.s.w;
    const uint32_t l = (uint32_t)lane_id();
    uint32_t wv[4], tot = 0;
    bool bad = false;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int i = (int)l + 64 * c;
        wv[c] = i < nw ? w[i] : 0u;
        bad |= wv[c] > 11;
        if (wv[c] && wv[c] <= 11) tot += 1u << (wv[c] - 1);
    }
    if (__ballot(bad)) return -1;
    const uint32_t total = wave_sum(tot);
    if (total == 0) return -1;
    const int maxbits = hb32(total) + 1;
    if (maxbits > 11) return -1;
    const uint32_t rest = (1u << maxbits) - total;
    if (rest & (rest - 1)) return -1;
    const uint32_t wl = hb32(rest) + 1;  // the last symbol's weight (nw <= 255, so it is in chunk nw / 64)
#pragma unroll
    for (int c = 0; c < 4; c++)
        if ((int)l + 64 * c == nw) wv[c] = wl;
    uint32_t pos[4] = {0, 0, 0, 0}, run = 0;
    const uint64_t lt = (1ull << l) - 1;
    for (uint32_t v = 1; v <= (uint32_t)maxbits; v++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint64_t m = __ballot(wv[c] == v);
            if (wv[c] == v) pos[c] = run + ((uint32_t)__popcll(m & lt) << (v - 1));
            run += (uint32_t)__popcll(m) << (v - 1);
        }
    const uint32_t size = 1u << maxbits, g = size >= 64 ? size >> 6 : 1u, u0 = l * g;
    uint16_t *huf = t.s.huf;
    for (uint32_t u = l; u < size; u += 64) huf[u] = 0xFFFF;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c = 0; c < 4; c++)
        if (wv[c]) huf[pos[c]] = (uint16_t)((l + 64 * c) | (uint32_t)(maxbits + 1 - (int)wv[c]) << 8);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t last = 0;  // (cell + 1) << 16 | entry of the segment's last first-cell
    if (u0 < size)
        for (uint32_t j = 0; j < g; j++) {
            const uint32_t e = huf[u0 + j];
            if (e != 0xFFFF) last = (u0 + j + 1) << 16 | e;
        }
    const uint32_t before = wave_prev_lane(wave_incl_scan_op(last, [](uint32_t x, uint32_t y) { return x > y ? x : y; }));
    uint32_t cur = before & 0xFFFF;
    if (u0 < size)
        for (uint32_t j = 0; j < g; j++) {
            const uint32_t e = huf[u0 + j];
            if (e != 0xFFFF) cur = e;
            else huf[u0 + j] = (uint16_t)cur;
        }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    *maxbits_out = maxbits;
    return 0;
}

SDB_DEV int huf_read(EntLds &t, const uint8_t *in, uint64_t n, int *maxbits, bool wide) {
    if (n < 1) return -1;
    const int hb = in[0];
    uint8_t *w = t.s.w;
    int nw = 0;
    if (hb >= 128) {
        nw = hb - 127;
        const int nb = (nw + 1) / 2;
        if ((uint64_t)nb + 1 > n) return -1;
        for (int i = 0; i < nw; i++) w[i] = (i & 1) ? (in[1 + i / 2] & 15) : (in[1 + i / 2] >> 4);
        if (wide && SDB_ZS_WHUF ? huf_from_weights_wide(t, nw, maxbits) : huf_from_weights(t, nw, maxbits)) return -1;
        return 1 + nb;
    }
    if ((uint64_t)hb + 1 > n || hb == 0) return -1;
    const uint8_t *p = in + 1;
    int nsym, al;
    const int used = fse_read_ncount(p, (uint64_t)hb, t.s.norm, &nsym, 255, 6, &al);
    if (used < 0) return -1;
    FseCell *ft = t.s.wt;
    if (wide ? fse_build_wide(ft, t.s.norm, t.s.next, nsym, al) : fse_build(ft, t.s.norm, t.s.next, nsym, al)) return -1;
    RevBits b;
    if (!b.init(p + used, hb - used)) return -1;
    uint32_t s1 = b.get(al), s2 = b.get(al);
    if (b.pos < 0) return -1;
    for (;;) {
        if (nw >= 255) return -1;
        const uint32_t c1 = fse_cell(ft, s1);
        w[nw++] = (uint8_t)c1;
        s1 = (c1 >> 16) + b.get((int)((c1 >> 8) & 0xFF));
        if (b.pos < 0) {
            if (nw >= 255) return -1;
            w[nw++] = (uint8_t)fse_cell(ft, s2);
            break;
        }
        if (nw >= 255) return -1;
        const uint32_t c2 = fse_cell(ft, s2);
        w[nw++] = (uint8_t)c2;
        s2 = (c2 >> 16) + b.get((int)((c2 >> 8) & 0xFF));
        if (b.pos < 0) {
            if (nw >= 255) return -1;
            w[nw++] = (uint8_t)fse_cell(ft, s1);
            break;
        }
    }
    if (wide && SDB_ZS_WHUF ? huf_from_weights_wide(t, nw, maxbits) : huf_from_weights(t, nw, maxbits)) return -1;
    return 1 + hb;
}

// one Huffman stream of cnt literals into out (nullptr: decode and discard)
SDB_DEV int huf_stream(const EntLds &t, int maxbits, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cnt) {
    RevBits b;
    if (!b.init(in, (int64_t)n)) return -1;
    for (uint64_t i = 0; i < cnt; i++) {
        const uint16_t e = t.s.huf[b.peek(maxbits)];
        if (out) out[i] = (uint8_t)e;
        b.pos -= e >> 8;
        if (b.pos < 0) return -1;
    }
    return b.pos == 0 ? 0 : -1;
}

__constant__ int16_t c_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                     2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t c_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t c_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t c_ll_base[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18,
                                       20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096,
                                       8192, 16384, 32768, 65536};
__constant__ uint8_t c_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                      1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t c_ml_base[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
                                       21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 37,
                                       39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051,
                                       4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t c_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11,
                                      12, 13, 14, 15, 16};

// the literal / match length codes (baseline, extra bits) into the wave's LDS: looked up once per
// sequence each, an LDS read instead of a global one on the sequence loop's dependent path.  Whole wave.
SDB_DEV void seq_codes_to_lds(EntLds &t) {
    for (uint32_t i = (uint32_t)lane_id(); i < 36 + 53; i += 64) {
        if (i < 36) t.s.llv[i] = c_ll_base[i] | (uint32_t)c_ll_bits[i] << 24;
        else t.s.mlv[i - 36] = c_ml_base[i - 36] | (uint32_t)c_ml_bits[i - 36] << 24;
    }
}

struct ZstdState {
    int al_ll, al_of, al_ml;
    bool have_ll, have_of, have_ml, have_huf;
    int huf_bits;
    uint32_t rep[3];
};

// one sequence table by mode: 0 predefined, 1 RLE, 2 FSE description, 3 repeat; bytes or -1
SDB_DEV int seq_table(EntLds &t, FseCell *ft, int *al, bool *have, int mode, const uint8_t *in, uint64_t n,
                      const int16_t *def, int ndef, int def_al, int max_sym, int max_al, bool wide) {
    auto build = [&](int ns, int a) {
        return wide ? fse_build_wide(ft, t.s.norm, t.s.next, ns, a) : fse_build(ft, t.s.norm, t.s.next, ns, a);
    };
    if (mode == 0) {
        for (int i = 0; i < ndef; i++) t.s.norm[i] = def[i];
        if (build(ndef, def_al)) return -1;
        *al = def_al;
        *have = true;
        return 0;
    }
    if (mode == 1) {
        if (n < 1 || in[0] > max_sym) return -1;
        ft[0].sym = in[0];
        ft[0].nb = 0;
        ft[0].base = 0;
        *al = 0;
        *have = true;
        return 1;
    }
    if (mode == 2) {
        int nsym, a;
        const int used = fse_read_ncount(in, n, t.s.norm, &nsym, max_sym, max_al, &a);
        if (used < 0 || build(nsym, a)) return -1;
        *al = a;
        *have = true;
        return used;
    }
    return *have ? 0 : -1;
}

// a compressed block; frame bytes o.p[fstart, o.len); `end`: the slot's end (run mode literal stage)
SDB_DEV int zstd_block(EntLds &t, ZstdState &z, const uint8_t *in, uint64_t n, EntOut &o, uint64_t fstart, uint64_t window) {
    if (n < 1) return -1;
    const int ltype = in[0] & 3, sf = (in[0] >> 2) & 3;
    uint64_t hdr, regen, csize = 0;
    int streams = 1;
    if (ltype < 2) {
        if (sf == 0 || sf == 2) {
            hdr = 1;
            regen = in[0] >> 3;
        } else if (sf == 1) {
            if (n < 2) return -1;
            hdr = 2;
            regen = (in[0] >> 4) + ((uint64_t)in[1] << 4);
        } else {
            if (n < 3) return -1;
            hdr = 3;
            regen = (in[0] >> 4) + ((uint64_t)in[1] << 4) + ((uint64_t)in[2] << 12);
        }
    } else {
        if (sf <= 1) {
            if (n < 3) return -1;
            const uint32_t h = in[0] | (uint32_t)in[1] << 8 | (uint32_t)in[2] << 16;
            hdr = 3;
            regen = (h >> 4) & 0x3FF;
            csize = (h >> 14) & 0x3FF;
            streams = sf == 0 ? 1 : 4;
        } else if (sf == 2) {
            if (n < 4) return -1;
            const uint32_t h = rd32b(in);
            hdr = 4;
            regen = (h >> 4) & 0x3FFF;
            csize = h >> 18;
            streams = 4;
        } else {
            if (n < 5) return -1;
            const uint64_t h = (uint64_t)rd32b(in) | (uint64_t)in[4] << 32;
            hdr = 5;
            regen = (h >> 4) & 0x3FFFF;
            csize = (h >> 22) & 0x3FFFF;
            streams = 4;
        }
    }
    if (regen > 128 * 1024) return -1;
    // the literal stage: the end of the slot (run mode), nothing (count mode)
    if (o.p && o.cap - o.len < regen) return -1;
    uint8_t *lit = o.p ? o.p + (o.cap - regen) : nullptr;
    uint64_t ip = hdr;
    if (ltype == 0) {
        if (ip + regen > n) return -1;
        if (lit) {  // the stage sits past every byte still to be written: a plain 16-byte copy
            const uint64_t n16 = regen & ~15ull, l = o.lane(), L = o.lanes();
            for (uint64_t i = 16 * l; i < n16; i += 16 * L) {
                uint4 w;
                __builtin_memcpy(&w, in + ip + i, 16);
                __builtin_memcpy(lit + i, &w, 16);
            }
            for (uint64_t i = n16 + l; i < regen; i += L) lit[i] = in[ip + i];
        }
        ip += regen;
    } else if (ltype == 1) {
        if (ip + 1 > n) return -1;
        if (lit)
            for (uint64_t i = o.lane(); i < regen; i += o.lanes()) lit[i] = in[ip];
        ip += 1;
    } else {
        if (ip + csize > n) return -1;
        const uint8_t *c = in + ip;
        uint64_t cn = csize;
        if (ltype == 2) {
            const int used = huf_read(t, c, cn, &z.huf_bits, o.wide);
            if (used < 0) return -1;
            z.have_huf = true;
            c += used;
            cn -= (uint64_t)used;
        } else if (!z.have_huf) {
            return -1;
        }
        if (streams == 1) {
            if (huf_stream(t, z.huf_bits, c, cn, lit, regen)) return -1;
        } else {
            if (cn < 10 || regen < 6) return -1;
            const uint64_t s1 = c[0] | (uint64_t)c[1] << 8, s2 = c[2] | (uint64_t)c[3] << 8, s3 = c[4] | (uint64_t)c[5] << 8;
            if (6 + s1 + s2 + s3 > cn) return -1;
            const uint64_t s4 = cn - 6 - s1 - s2 - s3, q = (regen + 3) / 4;
            const uint8_t *p = c + 6;
            if (o.wide) {  // lane l decodes stream l & 3 (four lanes per stream store the same bytes)
                const uint32_t j = (uint32_t)lane_id() & 3;
                const uint64_t off = j == 0 ? 0 : j == 1 ? s1 : j == 2 ? s1 + s2 : s1 + s2 + s3;
                const uint64_t sz = j == 0 ? s1 : j == 1 ? s2 : j == 2 ? s3 : s4;
                const int r = huf_stream(t, z.huf_bits, p + off, sz, lit ? lit + j * q : nullptr, j < 3 ? q : regen - 3 * q);
                if (__ballot(r != 0)) return -1;
            } else if (huf_stream(t, z.huf_bits, p, s1, lit, q) ||
                       huf_stream(t, z.huf_bits, p + s1, s2, lit ? lit + q : nullptr, q) ||
                       huf_stream(t, z.huf_bits, p + s1 + s2, s3, lit ? lit + 2 * q : nullptr, q) ||
                       huf_stream(t, z.huf_bits, p + s1 + s2 + s3, s4, lit ? lit + 3 * q : nullptr, regen - 3 * q)) {
                return -1;
            }
        }
        ip += csize;
    }
    if (ip >= n) return -1;
    uint64_t nseq = in[ip++];
    if (nseq >= 128) {
        if (nseq < 255) {
            if (ip >= n) return -1;
            nseq = ((nseq - 128) << 8) + in[ip++];
        } else {
            if (ip + 2 > n) return -1;
            nseq = in[ip] + ((uint64_t)in[ip + 1] << 8) + 0x7F00;
            ip += 2;
        }
    }
    uint64_t lp = 0;
    const uint64_t block_start = o.len;
    if (nseq > 0) {
        if (ip >= n) return -1;
        const int modes = in[ip++];
        if (modes & 3) return -1;
        int u = seq_table(t, t.s.ll, &z.al_ll, &z.have_ll, modes >> 6, in + ip, n - ip, c_ll_def, 36, 6, 35, 9, o.wide);
        if (u < 0) return -1;
        ip += (uint64_t)u;
        u = seq_table(t, t.s.of, &z.al_of, &z.have_of, (modes >> 4) & 3, in + ip, n - ip, c_of_def, 29, 5, 31, 8, o.wide);
        if (u < 0) return -1;
        ip += (uint64_t)u;
        u = seq_table(t, t.s.ml, &z.al_ml, &z.have_ml, (modes >> 2) & 3, in + ip, n - ip, c_ml_def, 53, 6, 52, 9, o.wide);
        if (u < 0) return -1;
        ip += (uint64_t)u;
        RevBits b;
        if (!b.init(in + ip, (int64_t)(n - ip))) return -1;
        uint32_t sll = b.get(z.al_ll), sof = b.get(z.al_of), sml = b.get(z.al_ml);
        uint32_t r0 = z.rep[0], r1 = z.rep[1], r2 = z.rep[2];
        for (uint64_t k = 0; k < nseq; k++) {
            const uint32_t cof = fse_cell(t.s.of, sof), cml = fse_cell(t.s.ml, sml),
                           cll = fse_cell(t.s.ll, sll);
            const uint32_t ofc = cof & 0xFF, mlc = cml & 0xFF, llc = cll & 0xFF;
            if (ofc > 31 || mlc > 52 || llc > 35) return -1;
            const uint32_t ofv = (1u << ofc) + b.get((int)ofc);
            const uint32_t mv = t.s.mlv[mlc], lv = t.s.llv[llc];
            const uint32_t ml = (mv & 0xFFFFFF) + b.get((int)(mv >> 24));
            const uint32_t ll = (lv & 0xFFFFFF) + b.get((int)(lv >> 24));
            if (k + 1 < nseq) {
                sll = (cll >> 16) + b.get((int)((cll >> 8) & 0xFF));
                sml = (cml >> 16) + b.get((int)((cml >> 8) & 0xFF));
                sof = (cof >> 16) + b.get((int)((cof >> 8) & 0xFF));
            }
            if (b.pos < 0) return -1;
            uint32_t off;
            if (ofv > 3) {
                off = ofv - 3;
                r2 = r1;
                r1 = r0;
                r0 = off;
            } else {
                const uint32_t idx = ll == 0 ? ofv : ofv - 1;
                if (idx == 0) {
                    off = r0;
                } else {
                    off = idx == 3 ? r0 - 1 : idx == 1 ? r1 : r2;
                    if (idx > 1) r2 = r1;
                    r1 = r0;
                    r0 = off;
                }
            }
            if (ll > regen - lp) return -1;
            // literals: the stage is at or past the write position (o <= end - R + lp), a forward copy is safe
            if (lit ? !o.copy_fwd(lit + lp, ll) : !o.copy(nullptr, ll)) return -1;
            lp += ll;
            if (off == 0 || off > o.len - fstart || off > window) return -1;
            if (!o.match(off, ml)) return -1;
        }
        z.rep[0] = r0;
        z.rep[1] = r1;
        z.rep[2] = r2;
        if (b.pos != 0) return -1;
    } else if (ip != n) {
        return -1;
    }
    if (lit ? !o.copy_fwd(lit + lp, regen - lp) : !o.copy(nullptr, regen - lp)) return -1;
    if (o.len - block_start > 128 * 1024) return -1;
    return 0;
}

// XXH64 of the frame's bytes (seed 0)
SDB_DEV uint64_t xrotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
SDB_DEV uint64_t xld64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}
SDB_DEV uint64_t xxh64_dev(const uint8_t *p, uint64_t n) {
    const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
    auto round = [&](uint64_t acc, uint64_t v) { return xrotl(acc + v * P2, 31) * P1; };
    const uint8_t *e = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        while (p + 32 <= e) {
            v1 = round(v1, xld64(p));
            v2 = round(v2, xld64(p + 8));
            v3 = round(v3, xld64(p + 16));
            v4 = round(v4, xld64(p + 24));
            p += 32;
        }
        h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
        h = (h ^ round(0, v1)) * P1 + P4;
        h = (h ^ round(0, v2)) * P1 + P4;
        h = (h ^ round(0, v3)) * P1 + P4;
        h = (h ^ round(0, v4)) * P1 + P4;
    } else {
        h = P5;
    }
    h += n;
    while (p + 8 <= e) {
        h ^= round(0, xld64(p));
        h = xrotl(h, 27) * P1 + P4;
        p += 8;
    }
    if (p + 4 <= e) {
        h ^= (uint64_t)rd32b(p) * P1;
        h = xrotl(h, 23) * P2 + P3;
        p += 4;
    }
    while (p < e) {
        h ^= (uint64_t)(*p++) * P5;
        h = xrotl(h, 11) * P1;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

SDB_DEV int zstd_decode(const uint8_t *in, uint64_t n, EntOut &o, EntLds &t) {
    uint64_t ip = 0;
    while (ip < n) {
        if (n - ip < 4) return -1;
        const uint32_t magic = rd32b(in + ip);
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (n - ip < 4) return -1;
            const uint32_t sz = rd32b(in + ip);
            ip += 4;
            if (n - ip < sz) return -1;
            ip += sz;
            continue;
        }
        if (magic != 0xFD2FB528u || ip >= n) return -1;
        const uint32_t fhd = in[ip++];
        const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
        if (fhd & 8) return -1;
        uint64_t window = 0;
        if (!single) {
            if (ip >= n) return -1;
            const uint32_t wd = in[ip++];
            const uint64_t base = 1ull << (10 + (wd >> 3));
            window = base + (base / 8) * (wd & 7);
        }
        const int did_len = did_flag == 3 ? 4 : did_flag;
        if (n - ip < (uint64_t)did_len) return -1;
        uint32_t did = 0;
        for (int i = 0; i < did_len; i++) did |= (uint32_t)in[ip + i] << (8 * i);
        ip += did_len;
        if (did) return -1;
        const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (n - ip < (uint64_t)fcs_len) return -1;
        uint64_t fcs = 0;
        for (int i = 0; i < fcs_len; i++) fcs |= (uint64_t)in[ip + i] << (8 * i);
        if (fcs_len == 2) fcs += 256;
        ip += fcs_len;
        if (single) window = fcs;
        if (window > (1ull << 27) + 1) return -1;
        ZstdState z{};
        z.rep[0] = 1;
        z.rep[1] = 4;
        z.rep[2] = 8;
        const uint64_t fstart = o.len;
        const uint64_t bmax = window < 128 * 1024 ? window : 128 * 1024;
        for (;;) {
            if (n - ip < 3) return -1;
            const uint32_t bh = in[ip] | (uint32_t)in[ip + 1] << 8 | (uint32_t)in[ip + 2] << 16;
            ip += 3;
            const int last = bh & 1, type = (bh >> 1) & 3;
            const uint64_t bs = bh >> 3;
            if (type == 3) return -1;
            if (type == 1) {
                if (bs > bmax || ip >= n) return -1;
                if (!o.fill(in[ip], bs)) return -1;
                ip += 1;
            } else {
                if (n - ip < bs || bs > bmax) return -1;
                if (type == 0) {
                    if (!o.copy(in + ip, bs)) return -1;
                } else if (zstd_block(t, z, in + ip, bs, o, fstart, window)) {
                    return -1;
                }
                ip += bs;
            }
            if (last) break;
        }
        if (fcs_len > 0 && o.len - fstart != fcs) return -1;
        if (checksum) {
            if (n - ip < 4) return -1;
            if (o.p && (uint32_t)xxh64_dev(o.p + fstart, o.len - fstart) != rd32b(in + ip)) return -1;
            ip += 4;
        }
    }
    return 0;
}

// The decoded size of a zstd stream from its frame headers alone: zstd::bulk::compress, the
// reference's encoder (format/sst.rs:590), writes Frame_Content_Size in every frame, so the plan walks
// frame and block headers (3 bytes per block, no entropy decoding).  -1 when a frame has no content
// size or a header is malformed: the caller then decodes the stream in count mode as before (and k_ent_run
// rejects a frame whose decoded size disagrees with its header, zstd_decode above).
SDB_DEV int zstd_frames_size(const uint8_t *in, uint64_t n, uint64_t *total) {
    uint64_t ip = 0, sum = 0;
    while (ip < n) {
        if (n - ip < 4) return -1;
        const uint32_t magic = rd32b(in + ip);
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
            if (n - ip < 4) return -1;
            const uint32_t sz = rd32b(in + ip);
            ip += 4;
            if (n - ip < sz) return -1;
            ip += sz;
            continue;
        }
        if (magic != 0xFD2FB528u || ip >= n) return -1;
        const uint32_t fhd = in[ip++];
        const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
        if (fhd & 8) return -1;
        const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (fcs_len == 0) return -1;
        const uint64_t hdr = (single ? 0 : 1) + (did_flag == 3 ? 4 : did_flag) + fcs_len;
        if (n - ip < hdr) return -1;
        ip += hdr - fcs_len;
        uint64_t fcs = 0;
        for (int i = 0; i < fcs_len; i++) fcs |= (uint64_t)in[ip + i] << (8 * i);
        if (fcs_len == 2) fcs += 256;
        ip += fcs_len;
        for (;;) {
            if (n - ip < 3) return -1;
            const uint32_t bh = in[ip] | (uint32_t)in[ip + 1] << 8 | (uint32_t)in[ip + 2] << 16;
            ip += 3;
            const uint32_t bt = (bh >> 1) & 3;
            const uint64_t csz = bt == 1 ? 1 : (bh >> 3);  // RLE: one stored byte
            if (bt == 3 || n - ip < csz) return -1;
            ip += csz;
            if (bh & 1) break;
        }
        if (checksum) {
            if (n - ip < 4) return -1;
            ip += 4;
        }
        // an untrusted header: a content size that would carry the sum past the output bound (or wrap it) is
        // malformed (a size its blocks do not produce is rejected by the run, zstd_decode)
        if (fcs > kEntMaxOut - sum) return -1;
        sum += fcs;
    }
    *total = sum;
    return 0;
}

// one codec per kernel instance (ZL: zlib, else zstd), so neither decoder's registers weigh on the other's
template <bool ZL>
SDB_DEV int ent_decode(const uint8_t *in, uint64_t n, EntOut &o, EntLds &t) {
    if constexpr (ZL) return zlib_decode(in, n, o, t.z);
    else return zstd_decode(in, n, o, t);
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
template <bool ZL>
__global__ __launch_bounds__(kEntThreads) void k_ent_plan(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    EntLds &t = *(EntLds *)(smem + 8 * 1024 + wave * kEntWaveLds);
    seq_codes_to_lds(t);
    __syncthreads();
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k <= a.nblocks; k += nw) {
        if (l != 0) continue;
        uint64_t slot = 0;
        if (k < a.nblocks) {
            const uint64_t s = a.block_off[k], e = a.block_off[k + 1];
            uint64_t fsz = 0;
            if (e >= s && e - s >= 4) {
                if (!ZL && !zstd_frames_size(a.blocks + s, e - s - 4, &fsz)) {
                    slot = fsz + 4;
                } else {
                    EntOut o{nullptr, 0, kEntMaxOut, false, false};
                    if (!ent_decode<ZL>(a.blocks + s, e - s - 4, o, t) && !o.bad) slot = o.len + 4;
                }
            }
        }
        a.slot[k] = slot;
    }
}

// crc32fast::hash of msg[0, n), every lane (tab: slicing tables in LDS)
SDB_DEV uint32_t ent_crc(const uint8_t *msg, uint64_t n, const uint32_t (*tab)[256]) {
    if (n >= 4) return wave_crc32_lds(msg, (uint32_t)n, tab);
    uint32_t x = 0xFFFFFFFFu;
    for (uint32_t q = 0; q < n; q++) x = tab[0][(x ^ msg[q]) & 0xFF] ^ (x >> 8);
    return x ^ 0xFFFFFFFFu;
}

template <bool ZL>
__global__ __launch_bounds__(kEntThreads) void k_ent_run(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    crc_slice_tables_to_lds((lu32 *)smem);
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    EntLds &t = *(EntLds *)(smem + 8 * 1024 + wave * kEntWaveLds);
    seq_codes_to_lds(t);
    __syncthreads();
    const uint32_t(*tab)[256] = (const uint32_t(*)[256])smem;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k < a.nblocks; k += nw) {
        const uint64_t s = a.block_off[k], e = a.block_off[k + 1], o = a.out_start[k];
        const uint64_t slot = a.out_start[k + 1] - o;
        int st = 0;
        uint64_t ol = 0;
        if (e < s || e - s < 4 || e - s > 0xFFFFFFFFull) {
            st = SDB_CORRUPT_BLOCK;
        } else {
            const uint64_t bl = e - s - 4;
            const uint8_t *in = a.blocks + s;
            const uint32_t stored = (uint32_t)in[bl] << 24 | (uint32_t)in[bl + 1] << 16 | (uint32_t)in[bl + 2] << 8 |
                                    (uint32_t)in[bl + 3];
            if (ent_crc(in, bl, tab) != stored) {
                st = SDB_CHECKSUM_MISMATCH;  // validate_checksum (format/sst.rs:1029-1038)
            } else if (slot == 0) {
                st = SDB_DECOMPRESSION_ERROR;
            } else if (o + slot > a.out_cap) {
                st = SDB_INVALID_ARGUMENT;
            } else {
                // every lane runs the decoder (same state; the copies spread over the lanes, EntOut::wide)
                EntOut out{a.out + o, 0, slot - 4, false, true};
                const int r = ent_decode<ZL>(in, bl, out, t) || out.bad ? SDB_DECOMPRESSION_ERROR : 0;
                st = __shfl(r, 0, 64);
                ol = (uint64_t)__shfl((long long)out.len, 0, 64);
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                if (!st) {
                    const uint32_t c = ent_crc(a.out + o, ol, tab);
                    if (l == 0) {
                        uint8_t *g = a.out + o;
                        g[ol] = (uint8_t)(c >> 24);
                        g[ol + 1] = (uint8_t)(c >> 16);
                        g[ol + 2] = (uint8_t)(c >> 8);
                        g[ol + 3] = (uint8_t)c;
                    }
                }
            }
        }
        if (l == 0) {
            a.out_end[k] = st ? o : o + ol + 4;
            if (st) atomicMin(a.err, (unsigned long long)((k << 8) | (uint64_t)st));
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Zlib has smaller code tables than zstd (ZTab, 4.3 KB), which leaves room in every wave's LDS for the
// compressed block itself: the bit reader's refills then hit LDS instead of HBM, one dependent round
// trip per 56 bits less.  Blocks over the stage are read from HBM as before.
constexpr uint32_t kZThreads = 1024;  // 16 waves per workgroup
constexpr uint32_t kZStage = 4352;
struct ZWave {
    ZTab t;
    uint8_t in[kZStage];
};
constexpr uint32_t kZWaveLds = (sizeof(ZWave) + 15) & ~15u;
constexpr uint32_t kZLds = 8 * 1024 + (kZThreads / 64) * kZWaveLds;
static_assert(kZLds <= 160 * 1024, "zlib decoder LDS");

// the block's bytes [g, g + n) staged in the wave's LDS (16-byte granules; the returned pointer is
// byte 0), or g itself when they do not fit.  Called by the whole wave.
SDB_DEV const uint8_t *zl_stage(const uint8_t *g, uint64_t n, uint8_t *buf) {
    const uintptr_t a0 = (uintptr_t)g & ~(uintptr_t)15;
    const uint32_t off = (uint32_t)((uintptr_t)g & 15);
    if (off + n + 15 > kZStage) return g;
    const uint32_t ng = (uint32_t)((off + n + 15) >> 4);
    for (uint32_t q = (uint32_t)lane_id(); q < ng; q += 64) ((uint4 *)buf)[q] = ((const uint4 *)a0)[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return buf + off;
}

__global__ __launch_bounds__(kZThreads) void k_zl_plan(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    ZWave &zw = *(ZWave *)(smem + 8 * 1024 + wave * kZWaveLds);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k <= a.nblocks; k += nw) {
        uint64_t slot = 0;
        if (k < a.nblocks) {
            const uint64_t s = a.block_off[k], e = a.block_off[k + 1];
            if (e >= s && e - s >= 4) {
                const uint8_t *in = zl_stage(a.blocks + s, e - s - 4, zw.in);
                if (l == 0) {
                    EntOut o{nullptr, 0, kEntMaxOut, false, false};
                    if (!zlib_decode(in, e - s - 4, o, zw.t) && !o.bad) slot = o.len + 4;
                }
            }
        }
        if (l == 0) a.slot[k] = slot;
        __builtin_amdgcn_wave_barrier();
    }
}

// The count-mode plan with several decoders per wave: lanes 0 .. D - 1 each decode their own block
// with their own code tables, reading the compressed bytes from HBM (the plan's speed tracks the number
// of decoders per CU, not where its input lives).
#ifndef SDB_ZL_PLAN_D
#define SDB_ZL_PLAN_D 5
#endif
constexpr uint32_t kZpD = SDB_ZL_PLAN_D, kZpTab = (sizeof(ZTab) + 15) & ~15u;
#ifndef SDB_ZL_WAVES
#define SDB_ZL_WAVES 14
#endif
constexpr uint32_t kZpThreads = 64 * SDB_ZL_WAVES;  // 70 decoders per workgroup (CU)
constexpr uint32_t kZpLds = (kZpThreads / 64) * kZpD * kZpTab;
static_assert(kZpLds <= 160 * 1024, "zlib plan LDS");
__global__ __launch_bounds__(kZpThreads) void k_zl_plan_multi(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    if (l >= kZpD) return;
    ZTab &t = *(ZTab *)(smem + (wave * kZpD + l) * kZpTab);
    const uint64_t ndec = (uint64_t)gridDim.x * (blockDim.x >> 6) * kZpD;
    const uint64_t n = a.nlist ? (*a.nlist < a.nblocks ? *a.nlist : a.nblocks) : a.nblocks;
    for (uint64_t k = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + wave) * kZpD + l; k <= a.nblocks; k += ndec) {
        uint64_t slot = 0;
        if (k < n) {
            const uint64_t b = a.list ? (uint64_t)a.list[k] : k;
            const uint64_t s = a.block_off[b], e = a.block_off[b + 1];
            if (e >= s && e - s >= 4) {
                EntOut o{nullptr, 0, kEntMaxOut, false, false};
                if (!zlib_decode(a.blocks + s, e - s - 4, o, t) && !o.bad) slot = o.len + 4;
            }
        }
        a.slot[k] = slot;
    }
}

// Adler-32 of p[0, n) by the whole wave (the sums of zlib_decode's wide path), in every lane
SDB_DEV uint32_t wave_adler32(const uint8_t *p, uint64_t n) {
    uint64_t sa = 0, sb = 0;
    for (uint64_t i = (uint64_t)lane_id(); i < n; i += 64) {
        const uint64_t b = p[i];
        sa += b;
        sb += (n - i) * b;
    }
    sa = wave_sum(sa);
    sb = wave_sum(sb);
    const uint32_t x = (uint32_t)((1 + sa) % 65521u), y = (uint32_t)((n % 65521u + sb % 65521u) % 65521u);
    return y << 16 | x;
}
// The same with lane l summing the 64-byte segments l, l + 64, ... from four 16-byte loads each, all in
// flight before the sums (k_zl_verify: one latency per 4 KiB instead of one per 64 bytes; more VGPRs)
SDB_DEV uint32_t wave_adler32_seg(const uint8_t *p, uint64_t n) {
    uint64_t sa = 0, sb = 0;
    for (uint64_t base = 64 * (uint64_t)lane_id(); base < n; base += 4096) {
        uint32_t w[16];
        if (base + 64 <= n && ((uintptr_t)(p + base) & 15) == 0) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint4 v = *(const uint4 *)(p + base + 16 * q);
                w[4 * q] = v.x;
                w[4 * q + 1] = v.y;
                w[4 * q + 2] = v.z;
                w[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                uint32_t x = 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (base + 4 * q + j < n) x |= (uint32_t)p[base + 4 * q + j] << (8 * j);
                w[q] = x;
            }
        }
        // bytes past n are 0: they add nothing to either sum
        uint32_t a32 = 0, b32 = 0;  // segment sums: sum b, sum (63 - i) b (< 2^23)
#pragma unroll
        for (int q = 0; q < 16; q++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t b = (w[q] >> (8 * j)) & 0xFF;
                a32 += b;
                b32 += (uint32_t)(63 - (4 * q + j)) * b;
            }
        // sum (n - i) b over the segment = (n - base - 63) * sum b + sum (63 - i) b
        sa += a32;
        sb += (uint64_t)(n - base - 63) * a32 + b32;
    }
    sa = wave_sum(sa);
    sb = wave_sum(sb);
    const uint32_t x = (uint32_t)((1 + sa) % 65521u), y = (uint32_t)((n % 65521u + sb % 65521u) % 65521u);
    return y << 16 | x;
}

// The run the same way: each wave takes kZpD blocks, checks their stored CRCs one after the other with
// the whole wave, lets lanes 0 .. kZpD - 1 decode one block each (copies and Adler-32 on that lane), then
// computes and appends the output CRCs with the whole wave again.
#ifndef SDB_ZL_WC
#define SDB_ZL_WC 1
#endif
#ifndef SDB_ZL_RUN_MULTI
#define SDB_ZL_RUN_MULTI 1
#endif
constexpr uint32_t kZrLds = 8 * 1024 + kZpLds;
static_assert(kZrLds <= 160 * 1024, "zlib run LDS");
template <bool>
__global__ __launch_bounds__(kZpThreads) void k_zl_run_multi(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    crc_slice_tables_to_lds((lu32 *)smem);
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    ZTab &t = *(ZTab *)(smem + 8 * 1024 + (wave * kZpD + (l < kZpD ? l : 0)) * kZpTab);
    __syncthreads();
    const uint32_t(*tab)[256] = (const uint32_t(*)[256])smem;
    const uint64_t ndec = (uint64_t)gridDim.x * (blockDim.x >> 6) * kZpD;
    // slot i decodes block blk(i) (the identity, or a decode-once pass's list); its output goes to
    // out_start[i] (out_start[blk(i)] when a.out_by_block: a list pass over the fixed slots)
    const uint64_t n = a.nlist ? (*a.nlist < a.nblocks ? *a.nlist : a.nblocks) : a.nblocks;
    auto blk = [&](uint64_t i) { return a.list ? (uint64_t)a.list[i] : i; };
    auto oix = [&](uint64_t i, uint64_t b) { return a.out_by_block ? b : i; };
    const bool optimistic = a.ovf_list != nullptr;
    for (uint64_t k0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + wave) * kZpD; k0 < n; k0 += ndec) {
        // 1. the stored CRCs (validate_checksum, format/sst.rs:1029-1038): lane j keeps block k0 + j's status
        int st = 0;
        for (uint32_t j = 0; j < kZpD; j++) {
            const uint64_t k = k0 + j;
            if (k >= n) break;
            const uint64_t b = blk(k);
            const uint64_t s = a.block_off[b], e = a.block_off[b + 1], o = a.out_start[oix(k, b)];
            const uint64_t slot = a.out_start[oix(k, b) + 1] - o;
            int sj = 0;
            if (e < s || e - s < 4 || e - s > 0xFFFFFFFFull) {
                sj = SDB_CORRUPT_BLOCK;
            } else {
                const uint64_t bl = e - s - 4;
                const uint8_t *g = a.blocks + s;
                const uint32_t stored = (uint32_t)g[bl] << 24 | (uint32_t)g[bl + 1] << 16 | (uint32_t)g[bl + 2] << 8 |
                                        (uint32_t)g[bl + 3];
                if (ent_crc(g, bl, tab) != stored) sj = SDB_CHECKSUM_MISMATCH;
                else if (slot == 0) sj = SDB_DECOMPRESSION_ERROR;
                else if (o + slot > a.out_cap) sj = SDB_INVALID_ARGUMENT;
            }
            if (l == j) st = sj;
        }
        // 2. lane j decodes block k0 + j (its Adler-32 checked below by the whole wave); optimistic slots: an
        //    output over the slot is not an error, the block is listed for its exact-size pass
        uint64_t ol = 0;
        uint32_t have = 0, want = 0, ovf = 0;
        const uint64_t kl = k0 + l;
        if (l < kZpD && kl < n && !st) {
            const uint64_t b = blk(kl);
            const uint64_t s = a.block_off[b], e = a.block_off[b + 1], o = a.out_start[oix(kl, b)];
            const uint64_t slot = a.out_start[oix(kl, b) + 1] - o;
            bool bad = false;
            int r;
            if (SDB_ZL_WC) {
                EntOutWC out{{a.out + o, 0, slot - 4, false, false, true, false, 0}, 0, 0};
                r = zlib_decode(a.blocks + s, e - s - 4, out, t);
                out.flush();
                bad = out.bad;
                ol = out.len;
                have = out.have_adler ? 1u : 0u;
                want = out.adler_want;
            } else {
                EntOut out{a.out + o, 0, slot - 4, false, false, true, false, 0};
                r = zlib_decode(a.blocks + s, e - s - 4, out, t);
                bad = out.bad;
                ol = out.len;
                have = out.have_adler ? 1u : 0u;
                want = out.adler_want;
            }
            st = r || bad ? SDB_DECOMPRESSION_ERROR : 0;
            if (optimistic && bad) {
                st = 0;
                ovf = 1;
            }
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        // 3. the output CRCs, trailers and out_end
        for (uint32_t j = 0; j < kZpD; j++) {
            const uint64_t k = k0 + j;
            if (k >= n) break;
            const uint64_t b = blk(k);
            int sj = __shfl(st, (int)j, 64);
            const uint64_t olj = (uint64_t)__shfl((long long)ol, (int)j, 64);
            const uint64_t o = a.out_start[oix(k, b)];
            if (__shfl((int)ovf, (int)j, 64)) {  // decode-once: the exact-size pass takes it
                if (l == 0) {
                    a.out_end[b] = o;
                    a.ovf_list[atomicAdd(a.ovf_count, 1ull)] = (uint32_t)b;
                }
                continue;
            }
            if (!sj && __shfl((int)have, (int)j, 64) && wave_adler32(a.out + o, olj) != (uint32_t)__shfl((int)want, (int)j, 64))
                sj = SDB_DECOMPRESSION_ERROR;
            if (!sj) {
                const uint32_t c = ent_crc(a.out + o, olj, tab);
                if (l == 0) {
                    uint8_t *gw = a.out + o;
                    gw[olj] = (uint8_t)(c >> 24);
                    gw[olj + 1] = (uint8_t)(c >> 16);
                    gw[olj + 2] = (uint8_t)(c >> 8);
                    gw[olj + 3] = (uint8_t)c;
                }
            }
            if (l == 0) {
                a.out_end[b] = sj ? o : o + olj + 4;
                if (sj) atomicMin(a.err, (unsigned long long)((b << 8) | (uint64_t)sj));
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// The wide pass (decode-once's first): every lane of the wave inflates a block of its own against the
// fixed code's tables, written once per workgroup into LDS, so the decoders per CU are bounded by waves,
// not by LDS (70 with a table set each).  It only decodes: each lane records its block's result in
// a.wres, and k_zl_verify then checks the stored CRC and the Adler-32 and appends the output CRC with one
// wave per block (the wave-wide checks of 64 blocks in a row would leave each wave waiting on memory
// 64 times over).  Blocks whose first deflate block is dynamic (or that meet one later), and streams too
// short for the bit reader's trailer rule, are listed (a.dyn_list) for k_zl_run_multi; blocks past their
// slot, as there, for the exact-size pass (a.ovf_list).
#ifndef SDB_ZL_WIDE_D
#define SDB_ZL_WIDE_D 64
#endif
constexpr uint32_t kZwD = SDB_ZL_WIDE_D;
constexpr uint32_t kZwThreads = 256, kZwRing = 256 * 64;  // a wave's history rings (EntOutRing)
constexpr uint32_t kZwLds = kZpTab + (kZwThreads / 64) * kZwRing;
static_assert(kZpTab % 16 == 0, "ZTab copies as 16-byte words");
// wres[2 b] = output length | code << 48 (kWrOk, kWrErr: the decode failed, kWrCap: the slot is past out_cap,
// kWrOther: another pass owns the block); wres[2 b + 1] = Adler-32 wanted | have << 32
enum : uint64_t { kWrOk = 0, kWrErr = 1, kWrCap = 2, kWrOther = 3 };
__global__ __launch_bounds__(kZwThreads) void k_zl_wide(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    ZTab &t = *(ZTab *)smem;
    zl_fixed_tables(t, threadIdx.x, blockDim.x);
    __syncthreads();
    const uint64_t n = a.nblocks;
    // kZwD decoding lanes per wave (the rest idle): fewer lanes, more waves to overlap the refill latency
    const uint64_t bstep = (uint64_t)gridDim.x * (blockDim.x >> 6) * kZwD;
    for (uint64_t b0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + wave) * kZwD; b0 < n; b0 += bstep) {
        const uint64_t b = l < kZwD ? b0 + l : n;
        bool dyn = false, ovf = false;
        if (b < n) {
            const uint64_t s = a.block_off[b], e = a.block_off[b + 1], o = a.out_start[b];
            const uint64_t slot = a.out_start[b + 1] - o;
            uint64_t code = kWrOk, ol = 0, adl = 0;
            if (e < s + 7 || e - s > 0xFFFFFFFFull || ((a.blocks[s + 2] >> 1) & 3) == 2) {
                dyn = true;
            } else if (o + slot > a.out_cap) {
                code = kWrCap;
            } else {
                EntOutRing out{{{a.out + o, 0, slot - 4, false, false, true, false, 0}, 0, 0},
                               (lu8 *)smem + kZpTab + wave * kZwRing + l};
#ifdef SDB_ZL_WIDE_INFLATE  // (diagnostic: inflate_raw's nested loops on the shared tables)
                const int r = zlib_decode<true>(a.blocks + s, e - s - 4, out, t);
#else
                const int r = zlib_decode_wide(a.blocks + s, e - s - 4, out, t);
#endif
                out.flush();
                if (r == 1) dyn = true;                // a dynamic block further into the stream
                else if (out.bad) ovf = true;          // past the slot: the exact-size pass
                else if (r) code = kWrErr;
                ol = out.len;
                adl = out.have_adler ? (1ull << 32) | out.adler_want : 0;
            }
            if (dyn || ovf) {
                code = kWrOther;
                a.out_end[b] = o;
            }
            a.wres[2 * b] = ol | code << 48;
            a.wres[2 * b + 1] = adl;
        }
        // the lists, one counter update per wave each
        const uint64_t dm = (uint64_t)__ballot(dyn), om = (uint64_t)__ballot(ovf), below = (1ull << l) - 1;
        if (dm) {
            unsigned long long base = 0;
            if (l == 0) base = atomicAdd(a.dyn_count, (unsigned long long)__builtin_popcountll(dm));
            base = (unsigned long long)__shfl((long long)base, 0, 64);
            if (dyn) a.dyn_list[base + __builtin_popcountll(dm & below)] = (uint32_t)b;
        }
        if (om) {
            unsigned long long base = 0;
            if (l == 0) base = atomicAdd(a.ovf_count, (unsigned long long)__builtin_popcountll(om));
            base = (unsigned long long)__shfl((long long)base, 0, 64);
            if (ovf) a.ovf_list[base + __builtin_popcountll(om & below)] = (uint32_t)b;
        }
    }
}

// One wave per block the wide pass decoded: the stored CRC (validate_checksum, format/sst.rs:1029-1038;
// it outranks the decode's status), the Adler-32 trailer, then the output CRC, out_end and the error word.
constexpr uint32_t kZvThreads = 256;
__global__ __launch_bounds__(kZvThreads) void k_zl_verify(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    crc_slice_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t(*tab)[256] = (const uint32_t(*)[256])smem;
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    for (uint64_t b = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; b < a.nblocks;
         b += (uint64_t)gridDim.x * (blockDim.x >> 6)) {
        const uint64_t w0 = a.wres[2 * b], code = w0 >> 48;
        if (code == kWrOther) continue;
        const uint64_t s = a.block_off[b], e = a.block_off[b + 1], o = a.out_start[b], ol = w0 & 0xFFFFFFFFFFFFull;
        const uint64_t bl = e - s - 4;
        const uint8_t *g = a.blocks + s;
        const uint32_t stored = (uint32_t)g[bl] << 24 | (uint32_t)g[bl + 1] << 16 | (uint32_t)g[bl + 2] << 8 | (uint32_t)g[bl + 3];
        int st = 0;
        if (ent_crc(g, bl, tab) != stored) st = SDB_CHECKSUM_MISMATCH;
        else if (code == kWrCap) st = SDB_INVALID_ARGUMENT;
        else if (code == kWrErr) st = SDB_DECOMPRESSION_ERROR;
        else {
            const uint64_t w1 = a.wres[2 * b + 1];
            if ((w1 >> 32) && wave_adler32_seg(a.out + o, ol) != (uint32_t)w1) st = SDB_DECOMPRESSION_ERROR;
        }
        if (!st) {
            const uint32_t c = ent_crc(a.out + o, ol, tab);
            if (l == 0) {
                uint8_t *gw = a.out + o;
                gw[ol] = (uint8_t)(c >> 24);
                gw[ol + 1] = (uint8_t)(c >> 16);
                gw[ol + 2] = (uint8_t)(c >> 8);
                gw[ol + 3] = (uint8_t)c;
            }
        }
        if (l == 0) {
            a.out_end[b] = st ? o : o + ol + 4;
            if (st) atomicMin(a.err, (unsigned long long)((b << 8) | (uint64_t)st));
        }
    }
}

__global__ __launch_bounds__(kZThreads) void k_zl_run(EntArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    crc_slice_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t(*tab)[256] = (const uint32_t(*)[256])smem;
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    ZWave &zw = *(ZWave *)(smem + 8 * 1024 + wave * kZWaveLds);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k < a.nblocks; k += nw) {
        const uint64_t s = a.block_off[k], e = a.block_off[k + 1], o = a.out_start[k];
        const uint64_t slot = a.out_start[k + 1] - o;
        int st = 0;
        uint64_t ol = 0;
        if (e < s || e - s < 4 || e - s > 0xFFFFFFFFull) {
            st = SDB_CORRUPT_BLOCK;
        } else {
            const uint64_t bl = e - s - 4;
            const uint8_t *g = a.blocks + s;
            const uint32_t stored = (uint32_t)g[bl] << 24 | (uint32_t)g[bl + 1] << 16 | (uint32_t)g[bl + 2] << 8 |
                                    (uint32_t)g[bl + 3];
            const uint8_t *in = zl_stage(g, bl, zw.in);
            if (ent_crc(in, bl, tab) != stored) {
                st = SDB_CHECKSUM_MISMATCH;  // validate_checksum (format/sst.rs:1029-1038)
            } else if (slot == 0) {
                st = SDB_DECOMPRESSION_ERROR;
            } else if (o + slot > a.out_cap) {
                st = SDB_INVALID_ARGUMENT;
            } else {
                // every lane runs the decoder (same state; the copies spread over the lanes, EntOut::wide)
                EntOut out{a.out + o, 0, slot - 4, false, true};
                const int r = zlib_decode(in, bl, out, zw.t) || out.bad ? SDB_DECOMPRESSION_ERROR : 0;
                st = __shfl(r, 0, 64);
                ol = (uint64_t)__shfl((long long)out.len, 0, 64);
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                if (!st) {
                    const uint32_t c = ent_crc(a.out + o, ol, tab);
                    if (l == 0) {
                        uint8_t *gw = a.out + o;
                        gw[ol] = (uint8_t)(c >> 24);
                        gw[ol + 1] = (uint8_t)(c >> 16);
                        gw[ol + 2] = (uint8_t)(c >> 8);
                        gw[ol + 3] = (uint8_t)c;
                    }
                }
            }
        }
        if (l == 0) {
            a.out_end[k] = st ? o : o + ol + 4;
            if (st) atomicMin(a.err, (unsigned long long)((k << 8) | (uint64_t)st));
        }
        __builtin_amdgcn_wave_barrier();
    }
}

static std::once_flag g_ent_once;
static hipError_t g_ent_attr = hipSuccess;
static void ent_attrs() {
    std::call_once(g_ent_once, [] {
        // (zlib takes its own kernels below; the <true> instances of the generic ones are never launched)
        for (const void *f : {(const void *)k_ent_plan<false>, (const void *)k_ent_run<false>})
            if (g_ent_attr == hipSuccess)
                g_ent_attr = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEntLds);
        if (g_ent_attr == hipSuccess)
            g_ent_attr = hipFuncSetAttribute((const void *)k_zl_plan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kZLds);
        if (g_ent_attr == hipSuccess)
            g_ent_attr = hipFuncSetAttribute((const void *)k_zl_run, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kZLds);
        if (g_ent_attr == hipSuccess)
            g_ent_attr = hipFuncSetAttribute((const void *)k_zl_plan_multi, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)kZpLds);
        if (g_ent_attr == hipSuccess)
            g_ent_attr = hipFuncSetAttribute((const void *)k_zl_run_multi<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)kZrLds);
        if (g_ent_attr == hipSuccess)
            g_ent_attr = hipFuncSetAttribute((const void *)k_zl_wide, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kZwLds);
    });
}
static uint32_t ent_grid(uint64_t nwaves, uint32_t threads = kEntThreads) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    uint64_t wgs = (nwaves + threads / 64 - 1) / (threads / 64);
    const uint64_t most = (uint64_t)(cus > 0 ? cus : 256);
    if (wgs > most) wgs = most;
    return (uint32_t)(wgs ? wgs : 1);
}

// the plan's per-block slots (the caller scans them)
hipError_t launch_ent_slots(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                            uint64_t *slot, hipStream_t st) {
    ent_attrs();
    if (g_ent_attr != hipSuccess) return g_ent_attr;
    EntArgs a{};
    a.codec = codec;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.slot = slot;
    if (codec == SDB_CODEC_ZLIB && kZpD > 1)
        hipLaunchKernelGGL(k_zl_plan_multi, dim3(ent_grid((nblocks + kZpD) / kZpD, kZpThreads)), dim3(kZpThreads), kZpLds, st, a);
    else if (codec == SDB_CODEC_ZLIB)
        hipLaunchKernelGGL(k_zl_plan, dim3(ent_grid(nblocks + 1, kZThreads)), dim3(kZThreads), kZLds, st, a);
    else
        hipLaunchKernelGGL(k_ent_plan<false>, dim3(ent_grid(nblocks + 1)), dim3(kEntThreads), kEntLds, st, a);
    return hipGetLastError();
}

hipError_t launch_ent_run(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks, uint8_t *out,
                          uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end, unsigned long long *err,
                          hipStream_t st) {
    ent_attrs();
    if (g_ent_attr != hipSuccess) return g_ent_attr;
    EntArgs a{};
    a.codec = codec;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.out = out;
    a.out_cap = out_cap;
    a.out_start = out_start;
    a.out_end = out_end;
    a.err = err;
    if (nblocks && codec == SDB_CODEC_ZLIB && SDB_ZL_RUN_MULTI)
        hipLaunchKernelGGL(k_zl_run_multi<false>, dim3(ent_grid((nblocks + kZpD - 1) / kZpD, kZpThreads)), dim3(kZpThreads), kZrLds,
                           st, a);
    else if (nblocks && codec == SDB_CODEC_ZLIB)
        hipLaunchKernelGGL(k_zl_run, dim3(ent_grid(nblocks, kZThreads)), dim3(kZThreads), kZLds, st, a);
    else if (nblocks)
        hipLaunchKernelGGL(k_ent_run<false>, dim3(ent_grid(nblocks)), dim3(kEntThreads), kEntLds, st, a);
    return hipGetLastError();
}

// zlib decode-once (launch_decompress_once, sdb_codec.hip): the optimistic run over fixed slots, which lists
// the blocks that overflowed theirs, and the exact plan + run over that list
bool zl_once_supported() { return SDB_ZL_RUN_MULTI && kZpD > 1; }

hipError_t launch_zl_once_slots(const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks, const uint32_t *list,
                                const unsigned long long *nlist, uint64_t *slot, hipStream_t st) {
    ent_attrs();
    if (g_ent_attr != hipSuccess) return g_ent_attr;
    EntArgs a{};
    a.codec = SDB_CODEC_ZLIB;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.slot = slot;
    a.list = list;
    a.nlist = nlist;
    hipLaunchKernelGGL(k_zl_plan_multi, dim3(ent_grid((nblocks + kZpD) / kZpD, kZpThreads)), dim3(kZpThreads), kZpLds, st, a);
    return hipGetLastError();
}

// mode 0: the per-decoder-table run; 1: the wide run (fixed-code blocks, the others to dyn_list)
hipError_t launch_zl_once_run(int mode, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks, uint8_t *out,
                              uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end, unsigned long long *err,
                              const uint32_t *list, const unsigned long long *nlist, bool out_by_block, uint32_t *ovf_list,
                              unsigned long long *ovf_count, uint32_t *dyn_list, unsigned long long *dyn_count,
                              uint64_t *wres, hipStream_t st) {
    ent_attrs();
    if (g_ent_attr != hipSuccess) return g_ent_attr;
    EntArgs a{};
    a.codec = SDB_CODEC_ZLIB;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.out = out;
    a.out_cap = out_cap;
    a.out_start = out_start;
    a.out_end = out_end;
    a.err = err;
    a.list = list;
    a.nlist = nlist;
    a.out_by_block = out_by_block;
    a.ovf_list = ovf_list;
    a.ovf_count = ovf_count;
    a.dyn_list = dyn_list;
    a.dyn_count = dyn_count;
    a.wres = wres;
    if (nblocks && mode == 1) {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint64_t most = 8ull * (cus > 0 ? cus : 256);
        uint64_t wgs = (nblocks + kZwD * (kZwThreads / 64) - 1) / (kZwD * (kZwThreads / 64));
        wgs = wgs < most ? wgs : most;
        hipLaunchKernelGGL(k_zl_wide, dim3((uint32_t)wgs), dim3(kZwThreads), kZwLds, st, a);
        uint64_t vgs = (nblocks + kZvThreads / 64 - 1) / (kZvThreads / 64);
        vgs = vgs < most ? vgs : most;
        hipLaunchKernelGGL(k_zl_verify, dim3((uint32_t)vgs), dim3(kZvThreads), 8 * 1024, st, a);
    }
    else if (nblocks)
        hipLaunchKernelGGL(k_zl_run_multi<false>, dim3(ent_grid((nblocks + kZpD - 1) / kZpD, kZpThreads)), dim3(kZpThreads),
                           kZrLds, st, a);
    return hipGetLastError();
}

}  // namespace sdb
