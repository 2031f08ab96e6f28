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

#define SIPROUND                                                                                   \
    do {                                                                                           \
        v0 += v1; v1 = __builtin_rotateleft64(v1, 13); v1 ^= v0; v0 = __builtin_rotateleft64(v0, 32); \
        v2 += v3; v3 = __builtin_rotateleft64(v3, 16); v3 ^= v2;                                   \
        v0 += v3; v3 = __builtin_rotateleft64(v3, 21); v3 ^= v0;                                   \
        v2 += v1; v1 = __builtin_rotateleft64(v1, 17); v1 ^= v2; v2 = __builtin_rotateleft64(v2, 32); \
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
//   k_bloom_bin   one workgroup per tile of kBinKeys keys: SipHash-1-3, the k probes, an LDS
//                 counting sort by slice; one global atomicAdd per (tile, slice) reserves a run in
//                 that slice's queue and the sorted probes are written run by run.
//   k_bloom_fill  one workgroup per slice of 2^sb bits: reads its queue (coalesced), ORs the probes
//                 into an LDS copy of the slice, writes the slice with plain stores.
// The queues hold the expected load + 8 sigma + one tile; a queue that would overflow (only for
// adversarial key sets) sets a flag and its slice is rebuilt by re-hashing every key.  The queue
// cursors and the flag are zeroed on the stream before the binning.  Deterministic (an OR).
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kBinThreads = 1024, kBinKeysPerThread = 4, kFillThreads = 1024;
constexpr uint32_t kBinMaxK = 15;  // probes per key (larger k: atomic path)
constexpr uint32_t kBinLds = 128 * 1024;
constexpr uint32_t kShards = 8;    // queues per slice: the tile's XCD-ish shard (blockIdx & 7)
constexpr uint32_t kFillUnroll = 8;  // 16-byte queue loads in flight per k_bloom_fill thread


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

// One binning tile (k_bloom_bin, or the bloom role of k_group): the (h0, d0) of each key come from
// the keys (FROM_HD false) or from hd[] (k_seg wrote them, FROM_HD true).  lds: dynamic LDS.
template <bool FROM_HD>
SDB_DEV void bloom_bin_tile(uint32_t tile, const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off,
                            const uint64_t *__restrict__ hd, uint64_t n, const BloomPlan &pl, const BloomQueues &q,
                            uint32_t *lds) {
    const uint32_t S = pl.nslices;
    uint32_t *hist = lds;                          // S: counts, then local run starts
    uint32_t *cur = hist + S;                      // S: local scatter cursors
    uint32_t *gbase = cur + S;                     // S: reserved queue positions
    uint32_t *sorted = gbase + S;                  // T * k probes, slice order
    __shared__ uint64_t s_w[17];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t k0 = (uint64_t)tile * pl.T;
    const uint64_t k1 = k0 + pl.T < n ? k0 + pl.T : n;
    const uint32_t nk = (uint32_t)(k1 - k0), np = nk * pl.k;
    const uint32_t shard = tile & (kShards - 1);
    for (uint32_t x = tid; x < S; x += nt) hist[x] = 0;
    // hashes stay in registers: key tid + j * nt of the tile
    uint32_t hh[kBinKeysPerThread], dd[kBinKeysPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kBinKeysPerThread; j++) {
        const uint32_t i = tid + j * nt;
        hh[j] = dd[j] = 0;
        if (i < nk) {
            if (FROM_HD) {
                const uint64_t v = hd[k0 + i];
                hh[j] = (uint32_t)v;
                dd[j] = (uint32_t)(v >> 32);
            } else {
                key_hd(key_bytes, key_off, k0 + i, pl, hh[j], dd[j]);
            }
        }
    }
#if defined(SDB_EXP_BIN_STAGE) && SDB_EXP_BIN_STAGE == 1
    if ((hh[0] ^ dd[1] ^ hh[2] ^ dd[3]) == 0x12345) q.cursor[0] = 7;  // keep the hashes live
    return;
#endif
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kBinKeysPerThread; j++)
        if (tid + j * nt < nk) probes_hd(hh[j], dd[j], pl.k, pl.m, [&](uint32_t p) { atomicAdd(&hist[p >> pl.sb], 1u); });
    __syncthreads();
#if defined(SDB_EXP_BIN_STAGE) && SDB_EXP_BIN_STAGE == 2
    return;
#endif
    // local run starts (exclusive scan) + one reservation per non-empty slice in this shard
    uint64_t carry = 0;
    for (uint32_t x0 = 0; x0 < S; x0 += nt) {
        const uint32_t x = x0 + tid;
        const uint32_t c = x < S ? hist[x] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(c, s_w, &tot);
        if (x < S) {
            gbase[x] = c ? atomicAdd(q.cursor + (uint64_t)x * kShards + shard, c) : 0;
            hist[x] = (uint32_t)(carry + ex);
            cur[x] = (uint32_t)(carry + ex);
        }
        carry += tot;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kBinKeysPerThread; j++)
        if (tid + j * nt < nk)
            probes_hd(hh[j], dd[j], pl.k, pl.m, [&](uint32_t p) { sorted[atomicAdd(&cur[p >> pl.sb], 1u)] = p; });
    __syncthreads();
#if defined(SDB_EXP_BIN_STAGE) && SDB_EXP_BIN_STAGE == 3
    return;
#endif
    // write the runs: sorted[x] belongs to slice sl = p >> sb at run position x - hist[sl]
    bool over = false;
    for (uint32_t x = tid; x < np; x += nt) {
        const uint32_t p = sorted[x], sl = p >> pl.sb;
        const uint32_t pos = gbase[sl] + (x - hist[sl]);
        if (pos < q.cap) q.queue[(sl * kShards + shard) * q.cap + pos] = p;  // < 2^32 probes (plan_fits)
        else over = true;
    }
    if (over) q.cursor[(uint64_t)S * kShards] = 1u;
}

// One bitmap slice (k_bloom_fill, or the bloom role of k_enum).  lds: dynamic LDS (2^sb bits).
SDB_DEV void bloom_fill_slice(uint32_t s, const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off,
                              const uint64_t *__restrict__ hd, uint64_t n, const BloomPlan &pl, const BloomQueues &q, uint8_t *bitmap, uint64_t bytes,
                              uint32_t *lds) {
    const uint32_t words = 1u << (pl.sb - 5);
    uint32_t *bits = lds;  // 2^sb bits
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    for (uint32_t x = tid; x < words; x += nt) bits[x] = 0;
    __syncthreads();
    const uint32_t lo = s << pl.sb;
#if defined(SDB_EXP_FILL_NOSET)
    auto set = [&](uint32_t p) { if (p == 0xFFFFFFFFu) bits[0] = p; };
#else
    auto set = [&](uint32_t p) { atomicOr(&bits[(p - lo) >> 5], 1u << (p & 31)); };
#endif
    if (q.cursor[(uint64_t)pl.nslices * kShards] == 0) {
        // the slice's kShards queues as one sequence of 16-byte units (each queue's < 4 tail probes
        // separately); every thread keeps kFillUnroll units in flight
        __shared__ uint32_t s_u[kShards + 1], s_cnt[kShards];
        if (tid < kShards) s_cnt[tid] = q.cursor[(uint64_t)s * kShards + tid];
        __syncthreads();
        if (tid == 0) {
            uint32_t u = 0;
            for (uint32_t sh = 0; sh < kShards; sh++) {
                s_u[sh] = u;
                u += s_cnt[sh] >> 2;
            }
            s_u[kShards] = u;
        }
        __syncthreads();
        const uint32_t nu = s_u[kShards];
        const uint4 *q4 = (const uint4 *)(q.queue + (uint64_t)s * kShards * q.cap);
        const uint32_t cap4 = q.cap >> 2;
        auto unit = [&](uint32_t u) -> const uint4 * {
            uint32_t sh = 0;
#pragma unroll
            for (uint32_t j = 1; j < kShards; j++) sh += u >= s_u[j];
            return q4 + sh * cap4 + (u - s_u[sh]);
        };
        for (uint32_t u0 = 0; u0 < nu; u0 += kFillUnroll * nt) {
            uint4 v[kFillUnroll];
#pragma unroll
            for (uint32_t j = 0; j < kFillUnroll; j++) {
                const uint32_t u = u0 + j * nt + tid;
                if (u < nu) v[j] = *unit(u);
            }
#pragma unroll
            for (uint32_t j = 0; j < kFillUnroll; j++) {
                if (u0 + j * nt + tid < nu) {
                    set(v[j].x);
                    set(v[j].y);
                    set(v[j].z);
                    set(v[j].w);
                }
            }
        }
        if (tid < kShards * 4) {  // tails: thread 4 sh + r takes probe r of queue sh's tail
            const uint32_t sh = tid >> 2, r = tid & 3, c = s_cnt[sh];
            if (r < (c & 3)) set(q.queue[((uint64_t)s * kShards + sh) * q.cap + (c & ~3u) + r]);
        }
    } else {
        // a queue overflowed: rebuild this slice from every key (hd: k_seg's (h0, d0), else hash)
        const uint32_t hi = lo + (1u << pl.sb) - 1;
        for (uint64_t i = tid; i < n; i += nt) {
            uint32_t h, d;
            if (hd) {
                const uint64_t v = hd[i];
                h = (uint32_t)v;
                d = (uint32_t)(v >> 32);
            } else {
                key_hd(key_bytes, key_off, i, pl, h, d);
            }
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
uint32_t bloom_queue_cap(uint64_t n, const BloomPlan &pl);
bool bloom_plan_fits(const BloomPlan &pl, uint64_t n);
uint64_t bloom_cursor_bytes(const BloomPlan &pl);
size_t bloom_bin_lds(const BloomPlan &pl);
size_t bloom_fill_lds(const BloomPlan &pl);
BloomQueues bloom_queues(void *ws, uint64_t n, const BloomPlan &pl);

}  // namespace sdb
