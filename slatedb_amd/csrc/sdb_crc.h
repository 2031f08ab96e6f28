// sdb_crc.h — the wave CRC32 of an LDS block image, shared by the encoder (k_emit) and the decoder.
//
// crc32fast 1.5 (CRC-32/ISO-HDLC, reflected 0xEDB88320) as slatedb stores it after every block
// (format/sst.rs:541-552, checked by validate_checksum format/sst.rs:1029-1038).  The tables live at
// LDS address 0 of the calling kernel (its only LDS is the dynamic region), so a lookup is
// `ds_read_b32 <byte offset>, offset:<table * 1024>` with no address add:
//   [0, 8 KiB)     slicing-by-8 tables
//   [8, 12 KiB)    x^256 byte tables (combine the two 32-byte chains of a segment)
//   [12, 36 KiB)   x^(512 * 2^s) byte tables, s = 0..5 (the six tree steps)
#pragma once
#include "sdb_device.h"

namespace sdb {

typedef __attribute__((address_space(3))) uint8_t lu8;
typedef __attribute__((address_space(3))) uint32_t lu32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lu128;

// 4 * byte SEL of w in one VALU op (SDWA operand select): the LDS byte offset of a table entry.
template <int SEL>
SDB_DEV uint32_t bytex4(uint32_t w) {
    uint32_t r;
    if constexpr (SEL == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
            : "=v"(r) : "v"(w));
    else if constexpr (SEL == 1)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
            : "=v"(r) : "v"(w));
    else if constexpr (SEL == 2)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
            : "=v"(r) : "v"(w));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
            : "=v"(r) : "v"(w));
    return r;
}
// k_emit keeps the tables at LDS address 0 (its only LDS is the dynamic region, checked at entry),
// so a lookup is ds_read_b32 <byte offset>, offset:<table * 1024> with no address add.
template <int T>
SDB_DEV uint32_t crc_tab(const lu32 *, uint32_t off4) {
    return *(const lu32 *)(uintptr_t)(T * 1024 + off4);
}
// slicing-by-8 step over the 8 message bytes (lo, hi), tables at LDS `tab` (8 x 256 u32)
SDB_DEV uint32_t crc_slice8_lds(uint32_t c, uint32_t lo, uint32_t hi, const lu32 *tab) {
    lo ^= c;
    const uint32_t x = crc_tab<7>(tab, bytex4<0>(lo)) ^ crc_tab<6>(tab, bytex4<1>(lo)) ^ crc_tab<5>(tab, bytex4<2>(lo));
    const uint32_t y = crc_tab<4>(tab, bytex4<3>(lo)) ^ crc_tab<3>(tab, bytex4<0>(hi)) ^ crc_tab<2>(tab, bytex4<1>(hi));
    const uint32_t z = crc_tab<1>(tab, bytex4<2>(hi)) ^ crc_tab<0>(tab, bytex4<3>(hi));
    return x ^ y ^ z;
}

// x^256 * c (the x^(8*32) shift of a CRC) from the 4 byte tables at LDS MB KiB (8: the standard layout)
template <int MB = 8>
SDB_DEV uint32_t crc_mul256_lds(uint32_t c) {
    return crc_tab<MB>(nullptr, bytex4<0>(c)) ^ crc_tab<MB + 1>(nullptr, bytex4<1>(c)) ^
           crc_tab<MB + 2>(nullptr, bytex4<2>(c)) ^ crc_tab<MB + 3>(nullptr, bytex4<3>(c));
}

// x^(8*64*2^s) * c from the 4 byte tables of tree step s (LDS TB KiB + s * 4 KiB; 12: standard layout)
template <int S, int TB = 12>
SDB_DEV uint32_t crc_tree_mul(uint32_t c) {
    return crc_tab<TB + 4 * S>(nullptr, bytex4<0>(c)) ^ crc_tab<TB + 1 + 4 * S>(nullptr, bytex4<1>(c)) ^
           crc_tab<TB + 2 + 4 * S>(nullptr, bytex4<2>(c)) ^ crc_tab<TB + 3 + 4 * S>(nullptr, bytex4<3>(c));
}

constexpr uint32_t kCrcTablesLds = 36 * 1024;

// Copy the tables into LDS [0, 36 KiB) (every thread of the workgroup; the caller synchronises).
SDB_DEV void crc_tables_to_lds(lu32 *crc) {
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) crc[q] = (&c_crc.t[0][0])[q];
    for (uint32_t q = threadIdx.x; q < 4 * 256; q += blockDim.x) crc[8 * 256 + q] = (&c_mul256.t[0][0])[q];
    for (uint32_t q = threadIdx.x; q < kTreeSteps * 4 * 256; q += blockDim.x) crc[12 * 256 + q] = (&g_tree.t[0][0][0])[q];
}
// Only the x^256 and tree tables, at LDS byte address `at` (28 KiB).
SDB_DEV void crc_combine_tables_to_lds(lu32 *at) {
    for (uint32_t q = threadIdx.x; q < 4 * 256; q += blockDim.x) at[q] = (&c_mul256.t[0][0])[q];
    for (uint32_t q = threadIdx.x; q < kTreeSteps * 4 * 256; q += blockDim.x) at[4 * 256 + q] = (&g_tree.t[0][0][0])[q];
}
// The slicing-by-8 tables alone (8 KiB) at `at`.
SDB_DEV void crc_slice_tables_to_lds(lu32 *at) {
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) at[q] = (&c_crc.t[0][0])[q];
}

// crc32fast::hash of the image [0, Lc), 4 <= Lc <= 4096, in every lane.  img: 16-byte aligned LDS,
// bytes [Lc, 64 * ceil(Lc / 64)) zero.  Segments are right-aligned on the lanes: lane l holds 64-byte
// segment l - (64 - nseg), two 32-byte slicing-by-8 chains each; lanes before the first segment hold 0
// (leading zero bytes leave a raw CRC unchanged).  Six pairwise tree steps combine them (lane 0 ends
// with the whole image), then the zero padding of the last segment is removed by x^(-8 t).
// fold_init: invert image bytes [0, 4) on the fly (crc32fast's 0xFFFFFFFF init); otherwise the caller
// has inverted the message's first four bytes in LDS (a message that starts past image byte 0).
SDB_DEV uint32_t wave_crc_image(const lu8 *img, uint32_t Lc, bool fold_init) {
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t nseg = (Lc + 63) >> 6;
    const lu32 *crc = (const lu32 *)(uintptr_t)0;
    uint32_t c = 0;
    {
        const int sg = (int)l - (64 - (int)nseg);
        if (sg >= 0) {
            const lu128 *src = (const lu128 *)(img + 64 * sg);
            u32x4 v0 = src[0], v1 = src[1], v2 = src[2], v3 = src[3];
            if (fold_init && sg == 0) v0.x = ~v0.x;  // crc32fast init 0xFFFFFFFF folded into bytes [0, 4)
            uint32_t ca = crc_slice8_lds(0, v0.x, v0.y, crc), cb = crc_slice8_lds(0, v2.x, v2.y, crc);
            ca = crc_slice8_lds(ca, v0.z, v0.w, crc);
            cb = crc_slice8_lds(cb, v2.z, v2.w, crc);
            ca = crc_slice8_lds(ca, v1.x, v1.y, crc);
            cb = crc_slice8_lds(cb, v3.x, v3.y, crc);
            ca = crc_slice8_lds(ca, v1.z, v1.w, crc);
            cb = crc_slice8_lds(cb, v3.z, v3.w, crc);
            c = crc_mul256_lds<>(ca) ^ cb;  // raw(seg) = raw(first 32) * x^256 + raw(last 32)
        }
    }
    // partner = lane + 2^s: DPP row_shl inside a row, then permlane16 / permlane32 swaps.  Lanes l with
    // l % 2^(s+1) != 0 hold nothing the tree still needs: their table lookups are masked off (inactive
    // lanes take no part in the LDS banking), 63 lanes' lookups in all instead of 384.
    {
        uint32_t p = dpp32<0x101>(c);
        if ((l & 1) == 0) c = crc_tree_mul<0>(c) ^ p;
        p = dpp32<0x102>(c);
        if ((l & 3) == 0) c = crc_tree_mul<1>(c) ^ p;
        p = dpp32<0x104>(c);
        if ((l & 7) == 0) c = crc_tree_mul<2>(c) ^ p;
        p = dpp32<0x108>(c);
        if ((l & 15) == 0) c = crc_tree_mul<3>(c) ^ p;
        p = (uint32_t)__builtin_amdgcn_permlane16_swap(c, c, false, false)[1];
        if ((l & 31) == 0) c = crc_tree_mul<4>(c) ^ p;
        p = (uint32_t)__builtin_amdgcn_permlane32_swap(c, c, false, false)[1];
        if (l == 0) c = crc_tree_mul<5>(c) ^ p;
    }
    const uint32_t u = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
    const uint32_t pad = (nseg << 6) - Lc;
    return gf_mul(c_seg.unpad[pad], u) ^ 0xFFFFFFFFu;
}

// Raw CRC of one 64-byte segment held in 16 little-endian dwords: two 32-byte slicing-by-8 chains
// combined by x^256 (the LDS tables of the k_emit layout).
SDB_DEV uint32_t crc_seg64_lds(const uint32_t (&m)[16]) {
    const lu32 *crc = (const lu32 *)(uintptr_t)0;
    uint32_t ca = crc_slice8_lds(0, m[0], m[1], crc), cb = crc_slice8_lds(0, m[8], m[9], crc);
    ca = crc_slice8_lds(ca, m[2], m[3], crc);
    cb = crc_slice8_lds(cb, m[10], m[11], crc);
    ca = crc_slice8_lds(ca, m[4], m[5], crc);
    cb = crc_slice8_lds(cb, m[12], m[13], crc);
    ca = crc_slice8_lds(ca, m[6], m[7], crc);
    cb = crc_slice8_lds(cb, m[14], m[15], crc);
    return crc_mul256_lds<>(ca) ^ cb;
}

// Combine the 64 lanes' segment CRCs (lane l's segment followed by those of lanes l+1 .. 63) into
// lane 0 by six pairwise tree steps; returns the wave-uniform result.  Tree tables at LDS TB KiB.
template <int TB = 12>
SDB_DEV uint32_t crc_tree_combine(uint32_t c) {
    const uint32_t l = (uint32_t)lane_id();
    // partner = lane + 2^s: DPP row_shl inside a row, then permlane16 / permlane32 swaps.  Lanes l with
    // l % 2^(s+1) != 0 hold nothing the tree still needs: their table lookups are masked off.
    uint32_t p = dpp32<0x101>(c);
    if ((l & 1) == 0) c = crc_tree_mul<0, TB>(c) ^ p;
    p = dpp32<0x102>(c);
    if ((l & 3) == 0) c = crc_tree_mul<1, TB>(c) ^ p;
    p = dpp32<0x104>(c);
    if ((l & 7) == 0) c = crc_tree_mul<2, TB>(c) ^ p;
    p = dpp32<0x108>(c);
    if ((l & 15) == 0) c = crc_tree_mul<3, TB>(c) ^ p;
    p = (uint32_t)__builtin_amdgcn_permlane16_swap(c, c, false, false)[1];
    if ((l & 31) == 0) c = crc_tree_mul<4, TB>(c) ^ p;
    p = (uint32_t)__builtin_amdgcn_permlane32_swap(c, c, false, false)[1];
    if (l == 0) c = crc_tree_mul<5, TB>(c) ^ p;
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
}

// crc32fast::hash of the message img[0, Lc), 4 <= Lc <= 4096, in every lane, with the 64-byte
// segments RIGHT-aligned to the message end: lane l holds [Lc - 64 (64 - l), +64).  The segment that
// straddles byte 0 reads the 64 bytes before img, which the caller keeps zero (leading zeros leave a
// raw CRC unchanged), so no trailing padding has to be divided out afterwards.  The caller has
// inverted message bytes [0, 4) in LDS (crc32fast's 0xFFFFFFFF init).  img: 4-byte aligned LDS.
// Reads are five 16-byte-aligned ds_read_b128 per lane (the same bank pattern as aligned segments),
// realigned by the wave-uniform byte shift Lc mod 16: a uniform branch on its dword part, one
// v_alignbyte per dword for the rest.  Lc must be wave-uniform.
template <int Q>
SDB_DEV void realign16(const uint32_t (&x)[20], uint32_t r, uint32_t (&m)[16]) {
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_alignbyte(x[i + Q + 1], x[i + Q], r);
}
SDB_DEV uint32_t wave_crc_image_ra(const lu8 *img, uint32_t Lc) {
    const uint32_t l = (uint32_t)lane_id();
    const int s = (int)Lc - 64 * (64 - (int)l);  // segment start (message coordinates)
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
    return crc_tree_combine<>(c) ^ 0xFFFFFFFFu;
}

// --- bank-replicated byte table (decode count pass) ------------------------------------------------
// The slicing-by-8 lookups above index a table by a data byte, so the 32 lanes of a ds_read_b32 group
// hit banks byte % 32 at random: ~3.7 LDS cycles per group instead of 1 (measured: 58 % of the count
// pass's LDS cycles were bank conflicts, and LDS was its bound).  Here table 0 (c = T[c & 0xFF] ^ c >> 8)
// is stored once per bank: entry i of copy b at byte 128 i + 4 b, and lane l reads copy l % 32, so every
// lookup is conflict-free.  32 KiB; one lookup and four VALU per byte.
constexpr uint32_t kCrcRepLds = 32 * 1024;

SDB_DEV void crc_rep_to_lds(lu32 *rep) {
    for (uint32_t q = threadIdx.x; q < 256 * 32; q += blockDim.x) rep[q] = c_crc.t[0][q >> 5];
}

template <uint32_t BASE>
SDB_DEV uint32_t crc_rep_step(uint32_t c, uint32_t lb) {
    uint32_t a;  // 128 * (c & 0xFF) in one op
    asm("v_lshlrev_b32_sdwa %0, 7, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(a) : "v"(c));
    return *(const lu32 *)(uintptr_t)((a | lb) + BASE) ^ (c >> 8);
}

// Raw CRC of one 64-byte segment (16 little-endian dwords): two 32-byte byte-at-a-time chains through
// the replicated table at LDS BASE, combined by x^256 (tables at LDS MB KiB; 8: the standard layout).
template <uint32_t BASE, int MB = 8>
SDB_DEV uint32_t crc_seg64_rep(const uint32_t (&m)[16]) {
    const uint32_t lb = ((uint32_t)lane_id() & 31) << 2;
    uint32_t ca = 0, cb = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        ca ^= m[i];
        cb ^= m[8 + i];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            ca = crc_rep_step<BASE>(ca, lb);
            cb = crc_rep_step<BASE>(cb, lb);
        }
    }
    return crc_mul256_lds<MB>(ca) ^ cb;
}

// wave_crc_image_ra with the per-segment CRC through the replicated table at LDS BASE; the x^256 and
// tree tables at LDS MB / TB KiB (8 / 12: the standard layout).
template <uint32_t BASE, int MB = 8, int TB = 12>
SDB_DEV uint32_t wave_crc_image_rep(const lu8 *img, uint32_t Lc) {
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
        c = crc_seg64_rep<BASE, MB>(m);
    }
    return crc_tree_combine<TB>(c) ^ 0xFFFFFFFFu;
}

}  // namespace sdb
