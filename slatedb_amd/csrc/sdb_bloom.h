// sdb_bloom.h — SipHash-1-3 filter hashing, probe sequence and the binned bitmap build, shared by
// the standalone bloom kernels (sdb_bloom.hip) and the fused encode kernels (sdb_encode.hip).
//
// filter_hash = SipHash-1-3 with a zero key over the raw key bytes (siphasher 1.0.3,
// slatedb/src/filter.rs:196-204); probes by enhanced double hashing (filter.rs:206-221); LSB-first
// bit order (filter.rs:223-233).
#pragma once
#include "sdb_device.h"
#include "sdb_encode.h"

namespace sdb {

// 64-bit rotate left by R (0 < R < 32) as two v_alignbit_b32 (the generic lowering is a 64-bit shift,
// a 32-bit shift and an or: one VALU more per rotate, 24 per hash)
template <int R>
SDB_DEV uint64_t rotl64(uint64_t x) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - R), nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    return ((uint64_t)nhi << 32) | nlo;
}
SDB_DEV uint64_t swap32(uint64_t x) { return (x << 32) | (x >> 32); }
#define SIPROUND                                                                 \
    do {                                                                         \
        v0 += v1; v1 = rotl64<13>(v1); v1 ^= v0; v0 = swap32(v0);               \
        v2 += v3; v3 = rotl64<16>(v3); v3 ^= v2;                                 \
        v0 += v3; v3 = rotl64<21>(v3); v3 ^= v0;                                 \
        v2 += v1; v1 = rotl64<17>(v1); v1 ^= v2; v2 = swap32(v2);               \
    } while (0)

// SipHash-1-3 of a 16-byte key whose bytes are the little-endian words m0, m1 (the D1 / config-4
// shape): two compression rounds, the length block (16 << 56), three finalisation rounds.
SDB_DEV uint64_t siphash13_16(uint64_t m0, uint64_t m1) {
    uint64_t v0 = 0x736f6d6570736575ULL, v1 = 0x646f72616e646f6dULL;
    uint64_t v2 = 0x6c7967656e657261ULL, v3 = 0x7465646279746573ULL;
    v3 ^= m0;
    SIPROUND;
    v0 ^= m0;
    v3 ^= m1;
    SIPROUND;
    v0 ^= m1;
    const uint64_t b = 16ull << 56;
    v3 ^= b;
    SIPROUND;
    v0 ^= b;
    v2 ^= 0xFF;
    SIPROUND;
    SIPROUND;
    SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

// x mod m for 32-bit x, m (Lemire, Kaser & Kurz: exact for every x and m >= 1), c = floor((2^64-1)/m)+1
SDB_DEV uint32_t fastmod_u32(uint32_t x, uint64_t c, uint32_t m) {
    const uint64_t low = c * x;  // mod 2^64
    const uint64_t t = (uint64_t)(uint32_t)low * m;
    return (uint32_t)(((uint64_t)(uint32_t)(low >> 32) * m + (t >> 32)) >> 32);
}

SDB_DEV uint64_t siphash13(const uint8_t *p, uint64_t n) {
    uint64_t v0 = 0x736f6d6570736575ULL, v1 = 0x646f72616e646f6dULL;
    uint64_t v2 = 0x6c7967656e657261ULL, v3 = 0x7465646279746573ULL;
    const uint64_t full = n & ~7ull;
    for (uint64_t i = 0; i < full; i += 8) {
        uint64_t m = load8(p + i, 8);
        v3 ^= m;
        SIPROUND;
        v0 ^= m;
    }
    uint64_t b = (n & 0xFF) << 56;
    const uint32_t rem = (uint32_t)(n & 7);
    if (rem) b |= load8(p + full, rem) & ((~0ull) >> (8 * (8 - rem)));
    v3 ^= b;
    SIPROUND;
    v0 ^= b;
    v2 ^= 0xFF;
    SIPROUND;
    SIPROUND;
    SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

// Enhanced double hashing over m bits (m < 2^32): h_0 = lo % m, d_0 = hi % m,
// d_i = (d_{i-1} + i) % m, h_{i+1} = (h_i + d_i) % m.  All intermediate values stay < 2m for
// i < m, so each step is one conditional subtract; tiny filters (m <= k) use the full modulo.
template <typename F>
SDB_DEV void for_each_probe(uint64_t hash, uint32_t k, uint32_t m, F f) {
    uint32_t h = (uint32_t)hash % m;
    uint32_t d = (uint32_t)(hash >> 32) % m;
    const bool small = m <= k;
    for (uint32_t i = 0; i < k; i++) {
        if (small) d = (uint32_t)(((uint64_t)d + i) % m);
        else {
            d += i;
            if (d >= m) d -= m;
        }
        if (!f(h)) return;
        uint32_t t = h + d;  // < 2m <= 2^33? m < 2^32 and h,d < m: use 64-bit to be safe
        uint64_t t64 = (uint64_t)h + d;
        h = t64 >= m ? (uint32_t)(t64 - m) : t;
    }
}

// ------------------------------------------------------------------------------------------------
// Build by binning probes into bitmap slices, then setting bits in LDS.  Random 32-bit atomics to
// HBM/L2 run at ~25 G/s on MI355X whatever their scope (scripts/probe.hip), i.e. ~136 us for the
// 3.47 M probes of one 64 MiB SST; LDS atomics are two orders of magnitude faster.
//   bin   one workgroup per tile of T keys (k_bloom_bin, or k_seg's chunk): SipHash-1-3, the k
//         probes, an LDS counting sort by slice.  The run of slice s goes to the tile's own slot
//         (s, tile) and its length to count[tile][s]: fixed places, so there is no global atomic
//         and nothing to initialise between calls.
//   fill  one workgroup per slice of 2^sb bits (k_bloom_fill, or k_enum's bloom role): every
//         tile's slot of the slice, ORed into an LDS copy of the slice, written with plain stores.
// A slot holds the expected run + 6 sigma + 16 probes; a longer run (adversarial key sets only) is
// recorded as kSlotOverflow and the fill rebuilds that slice from every key.  Deterministic (an OR).
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kBinThreads = 1024, kBinKeysPerThread = 4, kFillThreads = 1024;
constexpr uint32_t kBinMaxK = 15;  // probes per key (larger k: atomic path)
constexpr uint32_t kBinLds = 128 * 1024;
constexpr uint32_t kSlotOverflow = 0xFFFFFFFFu;
constexpr uint32_t kNoProbe = 0xFFFFFFFFu;  // never a probe: m < 2^32

// (h0, d0) of the enhanced double hashing for one key: h0 = lo % m, d0 = hi % m
SDB_DEV uint64_t key_hash(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t i) {
    const uint64_t ko = key_off[i], len = key_off[i + 1] - ko;
    if (len == 16 && (ko & 7) == 0) {
        const uint64_t *w = (const uint64_t *)(key_bytes + ko);
        return siphash13_16(w[0], w[1]);
    }
    return siphash13(key_bytes + ko, len);
}
SDB_DEV void key_hd(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t i, const BloomPlan &pl, uint32_t &h0,
                    uint32_t &d0) {
    const uint64_t h = key_hash(key_bytes, key_off, i);
    h0 = fastmod_u32((uint32_t)h, pl.mmod, pl.m);
    d0 = fastmod_u32((uint32_t)(h >> 32), pl.mmod, pl.m);
}
// the probes of for_each_probe from (h0, d0)
template <typename F>
SDB_DEV void probes_hd(uint32_t h, uint32_t d, uint32_t k, uint32_t m, F f) {
    if (m > k && m <= 0x80000000u) {
        // h + d, d + i < 2m <= 2^32: x mod m = min(x, x - m) in u32 (x - m wraps above x when x < m)
        for (uint32_t i = 0; i < k; i++) {
            d += i;
            const uint32_t dm = d - m;
            d = dm < d ? dm : d;
            f(h);
            h += d;
            const uint32_t hm = h - m;
            h = hm < h ? hm : h;
        }
        return;
    }
    const bool small = m <= k;
    for (uint32_t i = 0; i < k; i++) {
        if (small) d = (uint32_t)(((uint64_t)d + i) % m);
        else {
            d += i;
            if (d >= m) d -= m;
        }
        f(h);
        const uint64_t t64 = (uint64_t)h + d;
        h = t64 >= m ? (uint32_t)(t64 - m) : (uint32_t)t64;
    }
}

// The probes of the lane's keys (probes_hd's fast path: m > K, m <= 2^31) binned into the slices' LDS buckets:
// every probe first, then all their bucket reservations in flight together, then the offsets -- instead of
// one LDS round trip per probe (bloom_bin_core's one-pass plan)
template <uint32_t KPT, uint32_t K>
SDB_DEV void bin_probes_batched(const uint32_t (&hh)[KPT], const uint32_t (&dd)[KPT], uint32_t nk, const BloomPlan &pl,
                                uint32_t cap, uint32_t *cnt, uint16_t *bkt) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x, mask = (1u << pl.sb) - 1;
    uint32_t pp[KPT][K], pos[KPT][K];
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
        uint32_t h = hh[j], d = dd[j];
#pragma unroll
        for (uint32_t i = 0; i < K; i++) {
            d += i;
            const uint32_t dm = d - pl.m;
            d = dm < d ? dm : d;
            pp[j][i] = h;
            h += d;
            const uint32_t hm = h - pl.m;
            h = hm < h ? hm : h;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
#pragma unroll
        for (uint32_t i = 0; i < K; i++) pos[j][i] = cap;
        if (tid + j * nt < nk) {
#pragma unroll
            for (uint32_t i = 0; i < K; i++) pos[j][i] = atomicAdd(&cnt[pp[j][i] >> pl.sb], 1u);
        }
    }
#ifndef SDB_EXP_BIN_NOWRITE
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++)
#pragma unroll
        for (uint32_t i = 0; i < K; i++)
            if (pos[j][i] < cap) bkt[__umul24(pp[j][i] >> pl.sb, cap) + pos[j][i]] = (uint16_t)(pp[j][i] & mask);
#endif
}

// Bin one tile whose keys' (h0, d0) are held in registers: key tid + j * blockDim.x of the tile in
// (hh[j], dd[j]), nk keys.  An LDS counting sort by slice (histogram, scan, scatter), then every
// slice's run is written to the tile's slot with consecutive lanes on consecutive words (coalesced;
// storing each probe straight to its slot measured 3x slower: one cache line per lane).  lds: >=
// bloom_bin_lds(pl) bytes.  Called by the whole workgroup (barriers inside).
template <uint32_t KPT>
SDB_DEV void bloom_bin_core(uint32_t tile, const uint32_t (&hh)[KPT], const uint32_t (&dd)[KPT], uint32_t nk,
                            const BloomPlan &pl, const BloomSlots &q, uint32_t *lds) {
    const uint32_t S = pl.nslices;
    if (pl.one_pass) {
        // every probe takes the next place of its slice's LDS bucket (cap u16 offsets, the slot's own
        // capacity: a longer run is an overflow either way), then each bucket is copied to its slot
        uint32_t *cnt = lds;                                   // S
        uint16_t *bkt = (uint16_t *)(lds + ((S + 3) & ~3u));   // S x cap, 16-byte aligned (cap: multiple of 32)
        const uint32_t tid = threadIdx.x, nt = blockDim.x, cap = q.cap, mask = (1u << pl.sb) - 1;
        for (uint32_t x = tid; x < S; x += nt) cnt[x] = 0;
        __syncthreads();
        const bool fast = pl.m > pl.k && pl.m <= 0x80000000u;
        if (fast && pl.k == 6) {  // the default plan: 10 bits per key -> (u16)(10 * 0.69) = 6 probes
            bin_probes_batched<KPT, 6>(hh, dd, nk, pl, cap, cnt, bkt);
        } else if (fast && pl.k == 7) {
            bin_probes_batched<KPT, 7>(hh, dd, nk, pl, cap, cnt, bkt);
        } else if (fast && pl.k == 5) {
            bin_probes_batched<KPT, 5>(hh, dd, nk, pl, cap, cnt, bkt);
        } else {
#pragma unroll
            for (uint32_t j = 0; j < KPT; j++)
                if (tid + j * nt < nk)
                    probes_hd(hh[j], dd[j], pl.k, pl.m, [&](uint32_t p) {
                        const uint32_t sl = p >> pl.sb, pos = atomicAdd(&cnt[sl], 1u);
#ifndef SDB_EXP_BIN_NOWRITE  // diagnostic: the atomics alone
                        if (pos < cap) bkt[__umul24(sl, cap) + pos] = (uint16_t)(p & mask);  // sl < 256: full-rate mul
#endif
                    });
        }
        __syncthreads();
#if defined(SDB_EXP_BIN_NOWRITE) || defined(SDB_EXP_BIN_NOCOPY)  // diagnostic: no slot copy-out (empty runs)
        for (uint32_t x = tid; x < S; x += nt) q.count[(uint64_t)tile * S + x] = cnt[x] == 0x7FFFFFFF ? 1 : 0;
        return;
#endif
        for (uint32_t x = tid; x < S; x += nt) {
            const uint32_t c = cnt[x];
            q.count[(uint64_t)tile * S + x] = c <= cap ? c : kSlotOverflow;
        }
        // each half-wave copies one bucket per step, 16 bytes (eight offsets) per lane: a wave moves two runs
        // of up to 256 offsets per load / store pair; kU steps' loads are issued before any store.  Whole
        // 64-byte granules (cap is a multiple of 32): the words past the run carry stale bucket bytes, which
        // the fill never reads
        const uint64_t stride = (uint64_t)pl.tiles * cap;
        uint16_t *slots = (uint16_t *)q.slot + (uint64_t)tile * cap;
        const uint32_t w = tid >> 6, nw = nt >> 6, l = tid & 63, hl = l & 31;
        const uint32_t o8 = 8 * hl < cap ? 8 * hl : 0;  // (inside the bucket)
        constexpr uint32_t kU = 3;
        for (uint32_t sl0 = 2 * w + (l >> 5); sl0 < S; sl0 += 2 * nw * kU) {
            uint32_t c[kU];
            uint4 v[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t sl = sl0 + u * 2 * nw, sc = sl < S ? sl : 0;
                const uint32_t c0 = sl < S ? cnt[sc] : 0;
                c[u] = c0 < cap ? c0 : cap;
                v[u] = *(const uint4 *)(bkt + __umul24(sc, cap) + o8);
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t sl = sl0 + u * 2 * nw;
                const uint32_t cg = (c[u] + 31) & ~31u;
                if (sl < S && 8 * hl < cg) *(uint4 *)(slots + sl * stride + 8 * hl) = v[u];
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {  // runs over 256 offsets (cap > 256)
                const uint32_t sl = sl0 + u * 2 * nw;
                if (sl >= S || c[u] <= 256) continue;
                const uint32_t *src = (const uint32_t *)(bkt + sl * cap);
                uint32_t *dst = (uint32_t *)(slots + sl * stride);
                for (uint32_t i = 2 * hl + 256; i < c[u]; i += 64) {
                    if (i + 1 < c[u]) dst[i >> 1] = src[i >> 1];
                    else ((uint16_t *)dst)[i] = (uint16_t)src[i >> 1];
                }
            }
        }
        return;
    }
    uint32_t *hist = lds;        // S: counts, then local run starts
    uint32_t *cur = hist + S;    // S: local scatter cursors
    uint32_t *sorted = cur + S;  // nk * k probes, slice order
    __shared__ uint64_t s_w[17];
    const uint32_t tid = threadIdx.x, nt = blockDim.x, np = nk * pl.k;
    for (uint32_t x = tid; x < S; x += nt) hist[x] = 0;
    __syncthreads();
    const bool fast = pl.k == 6 && pl.m > pl.k && pl.m <= 0x80000000u;  // the default plan (10 bits per key)
    uint32_t pp[KPT][6];  // (fast) the probes of the lane's keys, generated once for both passes
    if (fast) {
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++) {
            uint32_t h = hh[j], d = dd[j];
#pragma unroll
            for (uint32_t i = 0; i < 6; i++) {  // probes_hd's fast path
                d += i;
                const uint32_t dm = d - pl.m;
                d = dm < d ? dm : d;
                pp[j][i] = h;
                h += d;
                const uint32_t hm = h - pl.m;
                h = hm < h ? hm : h;
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++)
            if (tid + j * nt < nk) {
#pragma unroll
                for (uint32_t i = 0; i < 6; i++) atomicAdd(&hist[pp[j][i] >> pl.sb], 1u);
            }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++)
            if (tid + j * nt < nk) probes_hd(hh[j], dd[j], pl.k, pl.m, [&](uint32_t p) { atomicAdd(&hist[p >> pl.sb], 1u); });
    }
    __syncthreads();
    // local run starts (exclusive scan); run lengths -> count[tile][s]
    uint64_t carry = 0;
    for (uint32_t x0 = 0; x0 < S; x0 += nt) {
        const uint32_t x = x0 + tid;
        const uint32_t c = x < S ? hist[x] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(c, s_w, &tot);
        if (x < S) {
            q.count[(uint64_t)tile * S + x] = c <= q.cap ? c : kSlotOverflow;
            hist[x] = (uint32_t)(carry + ex);
            cur[x] = (uint32_t)(carry + ex);
        }
        carry += tot;
    }
    __syncthreads();
    if (fast) {  // every cursor reservation of the lane in flight together, then the stores
        uint32_t pos[KPT][6];
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++) {
#pragma unroll
            for (uint32_t i = 0; i < 6; i++) pos[j][i] = ~0u;
            if (tid + j * nt < nk) {
#pragma unroll
                for (uint32_t i = 0; i < 6; i++) pos[j][i] = atomicAdd(&cur[pp[j][i] >> pl.sb], 1u);
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++)
#pragma unroll
            for (uint32_t i = 0; i < 6; i++)
                if (pos[j][i] != ~0u) sorted[pos[j][i]] = pp[j][i];
    } else {
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++)
            if (tid + j * nt < nk)
                probes_hd(hh[j], dd[j], pl.k, pl.m, [&](uint32_t p) { sorted[atomicAdd(&cur[p >> pl.sb], 1u)] = p; });
    }
    __syncthreads();
    // write the runs: sorted[x] belongs to slice sl = p >> sb at run position x - hist[sl]
    const uint64_t stride = (uint64_t)pl.tiles * q.cap;
    if (pl.sb <= 16) {  // u16 offsets inside the slice
        uint16_t *slots = (uint16_t *)q.slot + (uint64_t)tile * q.cap;
        const uint32_t mask = (1u << pl.sb) - 1;
        for (uint32_t x = tid; x < np; x += nt) {
            const uint32_t p = sorted[x], sl = p >> pl.sb;
            const uint32_t pos = x - hist[sl];
            if (pos < q.cap) slots[sl * stride + pos] = (uint16_t)(p & mask);
        }
    } else {
        uint32_t *slots = q.slot + (uint64_t)tile * q.cap;
        for (uint32_t x = tid; x < np; x += nt) {
            const uint32_t p = sorted[x], sl = p >> pl.sb;
            const uint32_t pos = x - hist[sl];
            if (pos < q.cap) slots[sl * stride + pos] = p;
        }
    }
}

// One binning tile of the standalone build: hash the tile's keys, then bin.
SDB_DEV void bloom_bin_tile(uint32_t tile, const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off,
                            uint64_t n, const BloomPlan &pl, const BloomSlots &q, uint32_t *lds) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t k0 = (uint64_t)tile * pl.T;
    const uint32_t nk = (uint32_t)((k0 + pl.T < n ? k0 + pl.T : n) - k0);
    uint32_t hh[kBinKeysPerThread], dd[kBinKeysPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kBinKeysPerThread; j++) {
        const uint32_t i = tid + j * nt;
        hh[j] = dd[j] = 0;
        if (i < nk) key_hd(key_bytes, key_off, k0 + i, pl, hh[j], dd[j]);
    }
    bloom_bin_core<kBinKeysPerThread>(tile, hh, dd, nk, pl, q, lds);
}

// One bitmap slice (k_bloom_fill, or the bloom role of k_enum).  lds: bloom_fill_lds(pl) bytes of
// dynamic LDS (the slice's bits, then the run length of every tile).
SDB_DEV void bloom_fill_slice(uint32_t s, const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off,
                              uint64_t n, const BloomPlan &pl, const BloomSlots &q, uint8_t *bitmap, uint64_t bytes,
                              uint32_t *lds) {
    const uint32_t words = 1u << (pl.sb - 5), T = pl.tiles;
    uint32_t *bits = lds;         // 2^sb bits
    uint32_t *cnt = bits + words;  // T: run length of each tile's slot
    __shared__ uint32_t s_over;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) s_over = 0;
    for (uint32_t x = tid; x < words; x += nt) bits[x] = 0;
    __syncthreads();
    for (uint32_t t = tid; t < T; t += nt) {
        const uint32_t c = q.count[(uint64_t)t * pl.nslices + s];
        cnt[t] = c;
        if (c == kSlotOverflow) s_over = 1;
    }
    __syncthreads();
    const uint32_t lo = s << pl.sb;
    auto set = [&](uint32_t p) { atomicOr(&bits[(p - lo) >> 5], 1u << (p & 31)); };
    if (!s_over && pl.sb <= 16) {
        // u16 offsets, 16 bytes (eight offsets) per lane: a wave reads four tiles' slots per load
        // instruction (lane group g = l / 16 takes a tile, lane gl its offsets 8 gl .. 8 gl + 7), four such
        // loads in flight per lane; a slot holds a run of ~T*k/S offsets (under 128 but for the tail of
        // the distribution: longer runs loop on).  Slots start 16-byte aligned (cap is a multiple of 8).
        const uint32_t w = tid >> 6, nw = nt >> 6, l = tid & 63, g = l >> 4, gl = l & 15;
        const uint16_t *base = (const uint16_t *)q.slot + (uint64_t)s * T * q.cap;
        auto set16 = [&](uint32_t o) { atomicOr(&bits[o >> 5], 1u << (o & 31)); };
        constexpr uint32_t kU = 4;
        for (uint32_t t0 = 4 * w; t0 < T; t0 += 4 * nw * kU) {
            uint4 v[kU];
            uint32_t c[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {  // unconditional loads (a clamped in-bounds slot when idle)
                const uint32_t t = t0 + u * 4 * nw + g;
                c[u] = t < T ? cnt[t] : 0;
                // lanes past the run read its first granule again (a line the group fetches anyway)
                const uint32_t tc = t < T ? t : 0, o = 8 * gl < c[u] && 8 * gl < q.cap ? 8 * gl : 0;
                v[u] = *(const uint4 *)(base + (uint64_t)tc * q.cap + o);
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t wv[4] = {v[u].x, v[u].y, v[u].z, v[u].w}, i0 = 8 * gl;
#pragma unroll
                for (uint32_t j = 0; j < 8; j++)
                    if (i0 + j < c[u]) set16((wv[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
                const uint32_t t = t0 + u * 4 * nw + g;
                for (uint32_t i = 128 + gl; i < c[u]; i += 16) set16(base[(uint64_t)t * q.cap + i]);
            }
        }
    } else if (!s_over) {
        // wave w takes tiles w, w + nw, ...; lane l reads probes l, l + 64, ... of a slot; four slots
        // in flight per wave
        const uint32_t w = tid >> 6, nw = nt >> 6, l = tid & 63;
        const uint32_t *base = q.slot + (uint64_t)s * T * q.cap;
        for (uint32_t t0 = w; t0 < T; t0 += 4 * nw) {
            uint32_t v[4][4];
#pragma unroll
            for (uint32_t u = 0; u < 4; u++) {
                const uint32_t t = t0 + u * nw;
                const uint32_t c = t < T ? cnt[t] : 0;
#pragma unroll
                for (uint32_t r = 0; r < 4; r++) {
                    const uint32_t i = l + 64 * r;
                    v[u][r] = i < c ? base[(uint64_t)t * q.cap + i] : kNoProbe;
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < 4; u++) {
#pragma unroll
                for (uint32_t r = 0; r < 4; r++)
                    if (v[u][r] != kNoProbe) set(v[u][r]);
                const uint32_t t = t0 + u * nw;  // runs longer than 256 probes (q.cap > 256)
                const uint32_t c = t < T ? cnt[t] : 0;
                for (uint32_t i = 256 + l; i < c; i += 64) set(base[(uint64_t)t * q.cap + i]);
            }
        }
    } else {
        // a slot overflowed: rebuild this slice from every key
        const uint32_t hi = lo + (1u << pl.sb) - 1;
        for (uint64_t i = tid; i < n; i += nt) {
            uint32_t h, d;
            key_hd(key_bytes, key_off, i, pl, h, d);
            probes_hd(h, d, pl.k, pl.m, [&](uint32_t p) {
                if (p >= lo && p <= hi) set(p);
            });
        }
    }
    __syncthreads();
    // slice bytes [lo/8, lo/8 + 2^sb/8) clipped to the bitmap
    const uint64_t b0 = (uint64_t)lo >> 3;
    const uint64_t b1 = (b0 + (words << 2)) < bytes ? b0 + (words << 2) : bytes;
    const uint64_t nfull = (b1 - b0) >> 2;
    for (uint64_t w = tid; w < nfull; w += nt) ((uint32_t *)(bitmap + b0))[w] = bits[w];
    for (uint64_t x = b0 + 4 * nfull + tid; x < b1; x += nt) {
        const uint64_t r = x - b0;
        bitmap[x] = (uint8_t)(bits[r >> 2] >> (8 * (r & 3)));
    }
}

// Host-side plan helpers (sdb_bloom.hip).
uint32_t bloom_slot_cap(const BloomPlan &pl);
bool bloom_plan_fits(const BloomPlan &pl);
size_t bloom_bin_lds(const BloomPlan &pl);
size_t bloom_fill_lds(const BloomPlan &pl);
uint64_t bloom_slots_bytes(const BloomPlan &pl);
BloomSlots bloom_slots(void *ws, const BloomPlan &pl);

}  // namespace sdb
