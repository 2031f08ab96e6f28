// sdb_device.h — device-side building blocks shared by the encode / bloom / decode kernels.
//
// gfx950 (CDNA4) only: 64-lane waves, byte work on VALU + LDS, no MFMA.  Nothing here is a port:
// the reference path is Rust on CPU (slatedb/src/format/*.rs, filter.rs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slatedb_amd.h"

#define SDB_DEV __device__ __forceinline__

namespace sdb {

constexpr int kWave = 64;

// ------------------------------------------------------------------------------------------------
// CRC-32/ISO-HDLC (crc32fast 1.5, reflected poly 0xEDB88320), tables built at compile time.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kPoly = 0xEDB88320u;

struct CrcTables {
    uint32_t t[8][256];
};
constexpr CrcTables make_crc_tables() {
    CrcTables r{};
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kPoly : (c >> 1);
        r.t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
        for (int s = 1; s < 8; s++) r.t[s][i] = (r.t[s - 1][i] >> 8) ^ r.t[0][r.t[s - 1][i] & 0xFF];
    return r;
}

// multmodp / x2nmodp (GF(2) arithmetic mod P in the reflected representation; "x^1" = 1<<30).
constexpr uint32_t gf_mul_c(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}
// x^(8*nbytes) mod P
constexpr uint32_t x8n_c(uint64_t nbytes) {
    uint32_t p = 1u << 31;  // x^0
    uint32_t sq = 1u << 30; // x^1
    uint64_t e = nbytes * 8;
    while (e) {
        if (e & 1) p = gf_mul_c(sq, p);
        sq = gf_mul_c(sq, sq);
        e >>= 1;
    }
    return p;
}
struct CrcShift64 {   // K[l] = x^(8*64*(63-l)): weight of lane l's 64-byte segment in a 4 KiB window
    uint32_t k[64];
    uint32_t window;  // x^(8*4096): shift of the running CRC past one full window
};
constexpr CrcShift64 make_shift64() {
    CrcShift64 r{};
    for (int l = 0; l < 64; l++) r.k[l] = x8n_c(64ull * (63 - l));
    r.window = x8n_c(4096);
    return r;
}

// Combine constants for CRCs computed over 64-byte segments of a 16-byte-aligned LDS image whose
// last segment is zero padded: seg[k] = x^(8*64*k) (weight of a segment followed by k segments),
// unpad[t] = x^(-8t) (removes t trailing zero bytes; x^-1 = (P + 1) / x, reflected 0xDB710641).
constexpr uint32_t kXInv = 0xDB710641u;
constexpr int kSegShifts = 80;
struct CrcSegShift {
    uint32_t seg[kSegShifts];
    uint32_t unpad[64];
};
constexpr CrcSegShift make_seg_shift() {
    CrcSegShift r{};
    for (int k = 0; k < kSegShifts; k++) r.seg[k] = x8n_c(64ull * k);
    uint32_t inv8 = 1u << 31;
    for (int q = 0; q < 8; q++) inv8 = gf_mul_c(kXInv, inv8);
    uint32_t p = 1u << 31;
    for (int t = 0; t < 64; t++) {
        r.unpad[t] = p;
        p = gf_mul_c(inv8, p);
    }
    return r;
}
static_assert(gf_mul_c(kXInv, 1u << 30) == (1u << 31), "x * x^-1 == 1");

// seg_mul[k][b][v] = x^(8*64*k) * (v << 8b) mod P: multiplies a CRC by the weight of k trailing
// 64-byte segments with 4 byte-table lookups.  Built by linearity from the 8 single-bit values.
struct CrcSegMul {
    uint32_t t[kSegShifts][4][256];
};
constexpr CrcSegMul make_seg_mul() {
    CrcSegMul r{};
    for (int k = 0; k < kSegShifts; k++) {
        uint32_t K = x8n_c(64ull * k);
        for (int b = 0; b < 4; b++) {
            uint32_t basis[8] = {};
            for (int i = 0; i < 8; i++) basis[i] = gf_mul_c(K, 1u << (8 * b + i));
            r.t[k][b][0] = 0;
            for (int v = 1; v < 256; v++) {
                int lo = __builtin_ctz(v);
                r.t[k][b][v] = r.t[k][b][v & (v - 1)] ^ basis[lo];
            }
        }
    }
    return r;
}

// mul256[b][v] = x^(8*32) * (v << 8b) mod P: shifts a CRC past 32 zero bytes (4 byte-table lookups).
struct CrcMul256 {
    uint32_t t[4][256];
};
constexpr CrcMul256 make_mul256() {
    CrcMul256 r{};
    const uint32_t K = x8n_c(32);
    for (int b = 0; b < 4; b++) {
        uint32_t basis[8] = {};
        for (int i = 0; i < 8; i++) basis[i] = gf_mul_c(K, 1u << (8 * b + i));
        r.t[b][0] = 0;
        for (int v = 1; v < 256; v++) r.t[b][v] = r.t[b][v & (v - 1)] ^ basis[__builtin_ctz(v)];
    }
    return r;
}

// tree[s][b][v] = x^(8*64*2^s) * (v << 8b) mod P, s = 0..5: the wave combine of 64 segment CRCs in
// 6 pairwise steps (left segment run shifted past a right run of 2^s 64-byte segments).
constexpr int kTreeSteps = 6;
struct CrcTree {
    uint32_t t[kTreeSteps][4][256];
};
constexpr CrcTree make_tree() {
    CrcTree r{};
    for (int s = 0; s < kTreeSteps; s++) {
        const uint32_t K = x8n_c(64ull << s);
        for (int b = 0; b < 4; b++) {
            uint32_t basis[8] = {};
            for (int i = 0; i < 8; i++) basis[i] = gf_mul_c(K, 1u << (8 * b + i));
            r.t[s][b][0] = 0;
            for (int v = 1; v < 256; v++) r.t[s][b][v] = r.t[s][b][v & (v - 1)] ^ basis[__builtin_ctz(v)];
        }
    }
    return r;
}

// Per translation unit (no relocatable device code needed).
static __device__ const CrcTree g_tree = make_tree();
static __constant__ CrcTables c_crc = make_crc_tables();
static __constant__ CrcShift64 c_shift = make_shift64();
static __constant__ CrcSegShift c_seg = make_seg_shift();
static __constant__ CrcMul256 c_mul256 = make_mul256();
struct CrcX8 {  // x^(8 r), r < 64: with c_seg.seg, the shift of a CRC past any n < 5120 bytes
    uint32_t t[64];
};
constexpr CrcX8 make_x8() {
    CrcX8 r{};
    for (int i = 0; i < 64; i++) r.t[i] = x8n_c((uint64_t)i);
    return r;
}
static __constant__ CrcX8 c_x8 = make_x8();
static __device__ const CrcSegMul g_seg_mul = make_seg_mul();
SDB_DEV uint32_t seg_shift_mul(uint32_t k, uint32_t c) {
    const uint32_t(*t)[256] = g_seg_mul.t[k];
    return t[0][c & 0xFF] ^ t[1][(c >> 8) & 0xFF] ^ t[2][(c >> 16) & 0xFF] ^ t[3][c >> 24];
}

// Runtime GF(2) multiply (branch-free, 32 steps).
SDB_DEV uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; i--) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
    }
    return p;
}
// A raw CRC shifted past n more message bytes (n < 5120): c * x^(8 n).
SDB_DEV uint32_t crc_shift_bytes(uint32_t c, uint32_t n) {
    return gf_mul(gf_mul(c_seg.seg[n >> 6], c_x8.t[n & 63]), c);
}

// ------------------------------------------------------------------------------------------------
// Byte helpers
// ------------------------------------------------------------------------------------------------
SDB_DEV uint32_t varint_len(uint32_t v) {  // utils.rs:638-645
    return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5;
}
SDB_DEV uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }

// Load 8 little-endian bytes at an arbitrary address p, of which only the first `need` (1..8) are
// required.  Reads only aligned 8-byte words that contain at least one required byte, so it never
// touches a page that holds no requested byte.  Bytes beyond `need` are unspecified.
SDB_DEV uint64_t load8(const uint8_t *p, uint32_t need) {
    uint32_t sh = (uint32_t)((uintptr_t)p & 7);
    const uint64_t *w = (const uint64_t *)(p - sh);  // pointer arithmetic keeps the address space
    uint64_t lo = w[0];
    if (sh == 0) return lo;
    uint64_t r = lo >> (8 * sh);
    if (need > 8 - sh) r |= w[1] << (8 * (8 - sh));
    return r;
}

// Longest common prefix of two byte strings (compute_prefix, block_v2.rs:52-75).
SDB_DEV uint32_t lcp_bytes(const uint8_t *a, uint32_t na, const uint8_t *b, uint32_t nb) {
    uint32_t n = na < nb ? na : nb, off = 0;
    while (off < n) {
        uint32_t need = n - off < 8 ? n - off : 8;
        uint64_t x = load8(a + off, need) ^ load8(b + off, need);
        if (need < 8) x &= (~0ull) >> (8 * (8 - need));
        if (x) return off + (uint32_t)(__builtin_ctzll(x) >> 3);
        off += need;
    }
    return n;
}

// ------------------------------------------------------------------------------------------------
// Wave primitives (wave64)
// ------------------------------------------------------------------------------------------------
SDB_DEV int lane_id() { return __lane_id(); }

// DPP (GFX9 data-parallel primitives): register-to-register lane moves on the VALU, no LDS round
// trip (ds_bpermute-based __shfl costs an LDS latency per step).
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143, kDppWaveShl1 = 0x130, kDppWaveShr1 = 0x138;

template <int CTRL, int ROWS = 0xF>
SDB_DEV uint32_t dpp32(uint32_t v) {  // lanes whose source is invalid / masked get 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS = 0xF>
SDB_DEV uint64_t dpp64(uint64_t v) {
    return (uint64_t)dpp32<CTRL, ROWS>((uint32_t)v) | ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(v >> 32)) << 32);
}
template <int CTRL, int ROWS = 0xF>
SDB_DEV uint32_t dpp(uint32_t v) { return dpp32<CTRL, ROWS>(v); }
template <int CTRL, int ROWS = 0xF>
SDB_DEV uint64_t dpp(uint64_t v) { return dpp64<CTRL, ROWS>(v); }

// Inclusive wave scan with an associative, identity-0 operator (row Kogge-Stone + row broadcasts).
template <typename T, typename Op>
SDB_DEV T wave_incl_scan_op(T v, Op op) {
    v = op(v, dpp<kDppRowShr1>(v));
    v = op(v, dpp<kDppRowShr2>(v));
    v = op(v, dpp<kDppRowShr4>(v));
    v = op(v, dpp<kDppRowShr8>(v));
    v = op(v, dpp<kDppRowBcast15, 0xA>(v));
    v = op(v, dpp<kDppRowBcast31, 0xC>(v));
    return v;
}
template <typename T>
SDB_DEV T wave_readlane(T v, int lane) {
    if constexpr (sizeof(T) == 8) {
        uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
        uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__builtin_amdgcn_readlane((int)v, lane);
    }
}
template <typename T>
SDB_DEV T wave_incl_scan(T v) {
    return wave_incl_scan_op(v, [](T x, T y) { return x + y; });
}
template <typename T>
SDB_DEV T wave_sum(T v) {  // every lane gets the total
    return wave_readlane(wave_incl_scan(v), 63);
}
SDB_DEV uint32_t wave_xor(uint32_t v) {
    return wave_readlane(wave_incl_scan_op(v, [](uint32_t x, uint32_t y) { return x ^ y; }), 63);
}
SDB_DEV uint32_t wave_max(uint32_t v) {
    return wave_readlane(wave_incl_scan_op(v, [](uint32_t x, uint32_t y) { return x > y ? x : y; }), 63);
}
// A raw buffer descriptor over [p, p + n) for range-checked loads / stores (an access past n is dropped,
// a load past n returns 0).  The inputs are readfirstlane'd so the compiler can see the descriptor is
// wave-uniform (it must be), otherwise it wraps every access in a waterfall loop.
SDB_DEV __amdgpu_buffer_rsrc_t wave_rsrc(const void *p, uint32_t n) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    const int nr = __builtin_amdgcn_readfirstlane((int)n);
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nr, 0x00020000);
}
// lane l gets lane l + 1's value (lane 63 gets 0)
template <typename T>
SDB_DEV T wave_next_lane(T v) {
    return dpp<kDppWaveShl1>(v);
}
// lane l gets lane l - 1's value (lane 0 gets 0)
template <typename T>
SDB_DEV T wave_prev_lane(T v) {
    return dpp<kDppWaveShr1>(v);
}

// ------------------------------------------------------------------------------------------------
// Error reporting: the reference stops at the first failing entry, so we keep min(entry<<8|code).
// ------------------------------------------------------------------------------------------------
SDB_DEV void report_error(unsigned long long *err_word, uint64_t entry, int code) {
    atomicMin(err_word, (unsigned long long)((entry << 8) | (uint64_t)code));
}

// ------------------------------------------------------------------------------------------------
// CRC of a byte range held in LDS, computed by one wave (64 lanes x 64-byte segments per 4 KiB
// window, right-aligned so every window but the first is full; zero prefix leaves a zero-init CRC
// unchanged).  The 0xFFFFFFFF init is folded in by inverting the first 4 message bytes.
// Returns crc32fast::hash(bytes) in every lane.  `tab` = slicing-by-8 tables in LDS.
// ------------------------------------------------------------------------------------------------
SDB_DEV uint32_t lds_read_u32_unaligned(const uint8_t *lds, uint32_t off) {
    const uint32_t *w = (const uint32_t *)(lds + (off & ~3u));
    uint32_t sh = off & 3;
    uint32_t lo = w[0];
    if (!sh) return lo;
    uint32_t hi = w[1];
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

SDB_DEV uint32_t crc_slice8(uint32_t c, uint32_t lo, uint32_t hi, const uint32_t (*tab)[256]) {
    lo ^= c;
    return tab[7][lo & 0xFF] ^ tab[6][(lo >> 8) & 0xFF] ^ tab[5][(lo >> 16) & 0xFF] ^ tab[4][lo >> 24] ^
           tab[3][hi & 0xFF] ^ tab[2][(hi >> 8) & 0xFF] ^ tab[1][(hi >> 16) & 0xFF] ^ tab[0][hi >> 24];
}

// Raw (zero-init, no xorout) CRC of msg[0, len) held in LDS, computed by one wave: 64 lanes x
// 64-byte segments per 4 KiB window, windows right-aligned so only the first is partial (a zero
// prefix leaves a zero-init CRC unchanged).  fold_init inverts message bytes [0,4), which turns the
// raw CRC into update(0xFFFFFFFF, msg).  Reads touch [msg - 3, msg + len + 7] at dword granularity;
// bytes outside [msg, msg + len) are masked.  Result is returned in every lane.
SDB_DEV uint32_t wave_crc_raw_lds(const uint8_t *msg, uint32_t len, const uint32_t (*tab)[256],
                                  bool fold_init) {
    const int l = lane_id();
    uint32_t nwin = (len + 4095) >> 12;
    uint32_t first = len - ((nwin - 1) << 12);  // bytes in the (right-aligned) first window
    uint32_t acc = 0;
    const uintptr_t base = (uintptr_t)msg;
    const uint8_t *b4 = (const uint8_t *)(base & ~(uintptr_t)3);
    const uint32_t bsh = (uint32_t)(base & 3);
    for (uint32_t w = 0; w < nwin; w++) {
        int64_t wend = (int64_t)first + ((int64_t)w << 12);
        int64_t seg0 = wend - 4096 + 64 * l;  // this lane's 64-byte segment start (message coords)
        uint32_t c = 0;
        if (seg0 + 64 > 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                int64_t s = seg0 + 8 * q;  // 8 bytes [s, s+8)
                uint32_t lo = 0, hi = 0;
                if (s + 8 > 0) {
                    int64_t sc = s < 0 ? 0 : s;
                    uint32_t off = bsh + (uint32_t)sc;
                    lo = lds_read_u32_unaligned(b4, off);
                    hi = lds_read_u32_unaligned(b4, off + 4);
                    uint64_t v = ((uint64_t)hi << 32) | lo;
                    if (s < 0) v <<= (uint32_t)(-s) * 8;  // zero the bytes before the message
                    if (fold_init && s < 4) {             // invert message bytes [0, 4)
                        int64_t from = -s;
                        uint64_t m = 0xFFFFFFFFull;
                        if (from >= 0) m <<= (uint32_t)from * 8;
                        else m >>= (uint32_t)(-from) * 8;
                        v ^= m;
                    }
                    lo = (uint32_t)v;
                    hi = (uint32_t)(v >> 32);
                }
                c = crc_slice8(c, lo, hi, tab);
            }
        }
        uint32_t win = wave_xor(gf_mul(c_shift.k[l], c));
        acc = (w == 0) ? win : (gf_mul(c_shift.window, acc) ^ win);
    }
    return acc;
}

// crc32fast::hash(msg[0, len)), len >= 4.
SDB_DEV uint32_t wave_crc32_lds(const uint8_t *msg, uint32_t len, const uint32_t (*tab)[256]) {
    return wave_crc_raw_lds(msg, len, tab, true) ^ 0xFFFFFFFFu;
}

// Raw CRC of one 64-byte segment held in registers (16 little-endian dwords, message order).
SDB_DEV uint32_t crc_seg64(const uint32_t (&w)[16], const uint32_t (*tab)[256]) {
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) c = crc_slice8(c, w[2 * q], w[2 * q + 1], tab);
    return c;
}

// LDS / global address-space helpers for LDS-DMA (global_load_lds_dword).
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
SDB_DEV uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)(const lds_u8 *)p; }
// dword at global `src` (any byte alignment) -> LDS byte address lds_base + 4 * lane
SDB_DEV void glds_dword(const uint8_t *src, uint32_t lds_base) {
    __builtin_amdgcn_global_load_lds((glb_void *)src, (lds_void *)(uintptr_t)lds_base, 4, 0, 0);
}

// Block-wide exclusive scan of u64 (blockDim.x <= 1024).  s_w: >= 17 u64 of LDS.
SDB_DEV uint64_t block_excl_scan_u64(uint64_t v, uint64_t *s_w, uint64_t *total) {
    const uint32_t tid = threadIdx.x, w = tid >> 6, nw = (blockDim.x + 63) >> 6;
    uint64_t inc = wave_incl_scan(v);
    if ((tid & 63) == 63 || tid == blockDim.x - 1) s_w[w] = inc;
    __syncthreads();
    if (tid == 0) {
        uint64_t c = 0;
        for (uint32_t q = 0; q < nw; q++) {
            uint64_t t = s_w[q];
            s_w[q] = c;
            c += t;
        }
        s_w[16] = c;
    }
    __syncthreads();
    uint64_t r = s_w[w] + inc - v;
    *total = s_w[16];
    __syncthreads();
    return r;
}

}  // namespace sdb
