// sdb_crc_mfma.h — the wave CRC32 of an LDS block image on the matrix cores (gfx950 MFMA, i8).
//
// A CRC is GF(2)-linear in its message bits, so the raw (zero-init) CRC of the 64-byte segments a wave
// holds (lane l: segment l of a right-aligned 4 KiB window, as wave_crc_image_ra) is a matrix product
// over GF(2): D[n][r] = sum_k W[n][k] * bit_k(segment pair r) mod 2.  v_mfma_i32_32x32x32_i8 computes
// the integer sum; its parity is the GF(2) product.  Operand lane maps (gfx950): lane l supplies
// A[row l&31][k = 16(l>>5) + j] and B[k = 16(l>>5) + j][col l&31], j = 0..15, so column r of B takes
// k 0..15 from lane r and k 16..31 from lane r + 32: one column is the PAIR of segments r and r + 32,
// 2048 bytes apart, and W's rows 0..15 carry the extra x^(8*2048) of the earlier one.
//   K-step t = 8g + b (g: 16-byte group of the segment, b: bit of the byte):
//     B (data):    lane's segment bytes 16g .. 16g+15 & (1 << b)  — the byte 2^b (b = 7: -128) or 0;
//     A (weights): bit n = l & 31 of W(h, byte 16g + j, bit b) * s(b), s(b) = 2^(7-b) (b = 0: -128), so
//                  every product of two set bits is +-128 and bit 7 of the sum is the parity.
//   32 K-steps, one accumulator: D[n][r] in lane r (rows n of its half) / lane r + 32 (the other half),
//   packed into a 32-bit word per pair, then pairs r = 0..31 combined by five tree steps (x^(8*64*2^s)).
// Against slicing-by-8 (wave_crc_image_ra): the 64 random-index ds_read_b32 per lane (bank conflicts:
// ~450 LDS cycles per 4 KiB block) become 32 conflict-free ds_read_b128 of the weights (128 cycles) and
// 32 MFMAs (the matrix pipe, otherwise idle in this byte work); the VALU count stays about the same.
#pragma once
#include "sdb_crc.h"

namespace sdb {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

// weights: [t = 8g + b][lane][j] int8, 32 KiB
struct CrcMfmaW {
    int8_t w[32][64][16];
};
// raw (zero-init) CRC register of a 64-byte segment whose only set bit is bit b of byte p
constexpr uint32_t crc_seg_bit_c(const CrcTables &T, uint32_t p, uint32_t b) {
    uint32_t c = T.t[0][1u << b];
    for (uint32_t q = p + 1; q < 64; q++) c = (c >> 8) ^ T.t[0][c & 0xFF];
    return c;
}
constexpr CrcMfmaW make_crc_mfma_w() {
    CrcMfmaW r{};
    const CrcTables T = make_crc_tables();
    const uint32_t shift2048 = x8n_c(2048);
    for (uint32_t p = 0; p < 64; p++)
        for (uint32_t b = 0; b < 8; b++) {
            const uint32_t w1 = crc_seg_bit_c(T, p, b), w0 = gf_mul_c(shift2048, w1);
            const uint32_t g = p >> 4, j = p & 15, t = 8 * g + b;
            const int8_t s = b == 0 ? (int8_t)-128 : (int8_t)(1 << (7 - b));
            for (uint32_t l = 0; l < 64; l++) {
                const uint32_t w = (l >> 5) ? w1 : w0, n = l & 31;
                r.w[t][l][j] = ((w >> n) & 1u) ? s : (int8_t)0;
            }
        }
    return r;
}
static __device__ const CrcMfmaW g_crc_mfma_w = make_crc_mfma_w();

constexpr uint32_t kCrcMfmaWLds = 32 * 1024;
// LDS layout of the MFMA CRC: [0, 32 KiB) weights, [32, 56 KiB) the six tree steps (crc_tree_mul<S, 32>)
constexpr uint32_t kCrcMfmaLds = kCrcMfmaWLds + kTreeSteps * 4 * 256 * 4;
constexpr int kCrcMfmaTreeKiB = 32;

// Copy the weights and tree tables into LDS [0, 56 KiB) (every thread of the workgroup; caller syncs).
SDB_DEV void crc_mfma_tables_to_lds(lu32 *at) {
    const uint32_t *w = (const uint32_t *)&g_crc_mfma_w.w[0][0][0];
    for (uint32_t q = threadIdx.x; q < kCrcMfmaWLds / 4; q += blockDim.x) at[q] = w[q];
    for (uint32_t q = threadIdx.x; q < kTreeSteps * 4 * 256; q += blockDim.x)
        at[kCrcMfmaWLds / 4 + q] = (&g_tree.t[0][0][0])[q];
}

// Raw CRC contribution of the 64 lanes' segments m[16] (lane l = segment l of a 4 KiB window, zeros where
// a lane holds none): sum_l raw(seg_l) * x^(8*64*(63-l)), wave-uniform.  Every lane must be active (MFMA).
// Weights at LDS byte address WB, tree tables at TB KiB.
template <uint32_t WB = 0, int TB = kCrcMfmaTreeKiB>
SDB_DEV uint32_t crc_segments_mfma(const uint32_t (&m)[16]) {
    const uint32_t l = (uint32_t)lane_id();
    i32x16 acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const lu128 *W = (const lu128 *)(uintptr_t)WB;
#pragma unroll
    for (int g = 0; g < 4; g++) {
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint32_t mk = 0x01010101u << b;
            const i32x4 d = {(int32_t)(m[4 * g] & mk), (int32_t)(m[4 * g + 1] & mk), (int32_t)(m[4 * g + 2] & mk),
                             (int32_t)(m[4 * g + 3] & mk)};
            const u32x4 w = W[(8 * g + b) * 64 + l];
            const i32x4 a = {(int32_t)w.x, (int32_t)w.y, (int32_t)w.z, (int32_t)w.w};
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, d, acc, 0, 0, 0);
        }
    }
    // lane l holds D[n][l & 31] for n = (i & 3) + 8 (i >> 2) + 4 (l >> 5), i = 0..15: parity = bit 7
    const uint32_t h4 = (l >> 5) * 4;
    uint32_t wd = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) wd |= (((uint32_t)acc[i] >> 7) & 1u) << ((i & 3) + 8 * (i >> 2));
    wd <<= h4;
    wd |= (uint32_t)__builtin_amdgcn_permlane32_swap(wd, wd, false, false)[1];  // the pair's two halves
    // pairs r = 0..31 (lanes 0..31): raw = sum_r D[r] * x^(8*64*(31-r)) by five tree steps
    uint32_t c = wd, p = dpp32<0x101>(c);
    if ((l & 1) == 0) c = crc_tree_mul<0, TB>(c) ^ p;
    p = dpp32<0x102>(c);
    if ((l & 3) == 0) c = crc_tree_mul<1, TB>(c) ^ p;
    p = dpp32<0x104>(c);
    if ((l & 7) == 0) c = crc_tree_mul<2, TB>(c) ^ p;
    p = dpp32<0x108>(c);
    if ((l & 15) == 0) c = crc_tree_mul<3, TB>(c) ^ p;
    p = (uint32_t)__builtin_amdgcn_permlane16_swap(c, c, false, false)[1];
    if ((l & 31) == 0) c = crc_tree_mul<4, TB>(c) ^ p;
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
}

// crc32fast::hash of the message img[0, Lc), 4 <= Lc <= 4096, right-aligned segments exactly as
// wave_crc_image_ra (the 64 bytes before img zero, message bytes [0, 4) inverted by the caller), on the
// matrix cores.  Lc wave-uniform; every lane active.
template <uint32_t WB = 0, int TB = kCrcMfmaTreeKiB>
SDB_DEV uint32_t wave_crc_image_mfma(const lu8 *img, uint32_t Lc) {
    const uint32_t l = (uint32_t)lane_id();
    const int s = (int)Lc - 64 * (64 - (int)l);  // segment start (message coordinates)
    uint32_t m[16];
    const int sg = s > -64 ? s : (int)(Lc & 15);  // lanes without a segment read (and drop) image bytes
    {
        const lu128 *w = (const lu128 *)(uintptr_t)(lds_addr((const void *)img) + (uint32_t)(sg - (int)(Lc & 15)));
        uint32_t x[20];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const u32x4 v = s > -64 ? w[i] : u32x4{0, 0, 0, 0};
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
    }
    return crc_segments_mfma<WB, TB>(m) ^ 0xFFFFFFFFu;
}

}  // namespace sdb
