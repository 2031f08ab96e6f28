// sdb_bloom.hip — bloom filter build / probe for gfx950.
//
// Replaces BloomFilterBuilder (slatedb/src/filter.rs:40-90) and BloomFilter::might_contain
// (filter.rs:124-136): filter_hash = SipHash-1-3 with a zero key over the raw key bytes
// (siphasher 1.0.3, filter.rs:196-204); probes by enhanced double hashing (filter.rs:206-221);
// LSB-first bit order (filter.rs:223-233).  Bit p of the byte-addressed bitmap is bit (p & 31) of the
// little-endian 32-bit word p >> 5, so setting it is one 32-bit atomicOr.
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

__global__ __launch_bounds__(256) void k_bloom_atomic(const uint8_t *__restrict__ key_bytes,
                                                      const uint64_t *__restrict__ key_off, uint64_t n,
                                                      uint32_t k, uint32_t m, uint32_t *bitmap) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t ko = key_off[i];
        uint64_t h = siphash13(key_bytes + ko, key_off[i + 1] - ko);
        for_each_probe(h, k, m, [&](uint32_t p) {
            atomicOr(bitmap + (p >> 5), 1u << (p & 31));
            return true;
        });
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

struct BloomQueues {
    uint32_t *cursor;  // nslices * kShards (+1: the overflow flag)
    uint32_t *queue;   // (nslices * kShards) x cap probes
    uint32_t cap;
};

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

__global__ __launch_bounds__(kBinThreads) void k_bloom_bin(const uint8_t *__restrict__ key_bytes,
                                                           const uint64_t *__restrict__ key_off, uint64_t n,
                                                           BloomPlan pl, BloomQueues q) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t S = pl.nslices;
    uint32_t *hist = lds;                          // S: counts, then local run starts
    uint32_t *cur = hist + S;                      // S: local scatter cursors
    uint32_t *gbase = cur + S;                     // S: reserved queue positions
    uint32_t *sorted = gbase + S;                  // T * k probes, slice order
    __shared__ uint64_t s_w[17];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t k0 = (uint64_t)blockIdx.x * pl.T;
    const uint64_t k1 = k0 + pl.T < n ? k0 + pl.T : n;
    const uint32_t nk = (uint32_t)(k1 - k0), np = nk * pl.k;
    const uint32_t shard = blockIdx.x & (kShards - 1);
    for (uint32_t x = tid; x < S; x += nt) hist[x] = 0;
    // hashes stay in registers: key tid + j * nt of the tile
    uint32_t hh[kBinKeysPerThread], dd[kBinKeysPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kBinKeysPerThread; j++) {
        const uint32_t i = tid + j * nt;
        hh[j] = dd[j] = 0;
        if (i < nk) key_hd(key_bytes, key_off, k0 + i, pl, hh[j], dd[j]);
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

__global__ __launch_bounds__(kFillThreads) void k_bloom_fill(const uint8_t *__restrict__ key_bytes,
                                                             const uint64_t *__restrict__ key_off, uint64_t n,
                                                             BloomPlan pl, BloomQueues q, uint8_t *bitmap,
                                                             uint64_t bytes) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t words = 1u << (pl.sb - 5);
    uint32_t *bits = lds;  // 2^sb bits
    const uint32_t s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
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
        // a queue overflowed: rebuild this slice from every key
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

__global__ __launch_bounds__(256) void k_bloom_query(const uint32_t *bitmap, uint32_t k, uint32_t m,
                                                     const uint8_t *__restrict__ key_bytes,
                                                     const uint64_t *__restrict__ key_off, uint64_t n,
                                                     uint8_t *result) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t r = 0;
        if (m) {
            uint64_t ko = key_off[i];
            uint64_t h = siphash13(key_bytes + ko, key_off[i + 1] - ko);
            r = 1;
            for_each_probe(h, k, m, [&](uint32_t p) {
                if (!((bitmap[p >> 5] >> (p & 31)) & 1u)) {
                    r = 0;
                    return false;
                }
                return true;
            });
        }
        result[i] = r;
    }
}

BloomPlan bloom_plan(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    BloomPlan pl{};
    pl.k = k ? k : 1;
    pl.m = (uint32_t)(bitmap_bytes * 8);
    // slices of 2^sb bits: at least 4 KiB, at most 64 KiB of LDS, and at most 256 of them
    pl.sb = 15;
    while (pl.sb < 19 && (((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb) > 256) pl.sb++;
    pl.nslices = (uint32_t)(((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb);
    if (pl.nslices == 0) pl.nslices = 1;
    // keys per binning tile: kBinKeysPerThread per thread, fewer when the sorted probes outgrow LDS
    uint32_t T = kBinThreads * kBinKeysPerThread;
    while (T > kBinThreads && 4ull * (3 * pl.nslices + (uint64_t)T * pl.k) > kBinLds) T -= kBinThreads;
    pl.T = T;
    pl.tiles = (uint32_t)((n + T - 1) / T);
    if (pl.tiles == 0) pl.tiles = 1;
    pl.mmod = pl.m ? ~0ull / pl.m + 1 : 0;
    return pl;
}

static uint32_t queue_cap(uint64_t n, const BloomPlan &pl) {
    // uniform probes: n k / (S shards) expected per queue; + 8 sigma + 1024
    const double mean = (double)n * pl.k / ((double)pl.nslices * kShards);
    uint64_t cap = (uint64_t)(mean + 8.0 * __builtin_sqrt(mean + 1.0)) + 1024;
    cap = (cap + 63) & ~63ull;
    return (uint32_t)(cap < 0xFFFFFFC0ull ? cap : 0xFFFFFFC0ull);
}

static uint32_t queue_cap(uint64_t n, const BloomPlan &pl);
static bool plan_fits(const BloomPlan &pl, uint64_t n) {
    return pl.k <= kBinMaxK && pl.sb <= 19 && pl.m >= 2 && 4ull * (3 * pl.nslices + (uint64_t)pl.T * pl.k) <= kBinLds &&
           (uint64_t)pl.nslices * kShards * queue_cap(n, pl) < (1ull << 32);
}

static uint64_t cursor_bytes(const BloomPlan &pl) { return ((uint64_t)(pl.nslices * kShards + 1) * 4 + 255) & ~255ull; }

uint64_t bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    BloomPlan pl = bloom_plan(n, k, bitmap_bytes);
    return cursor_bytes(pl) + (uint64_t)pl.nslices * kShards * queue_cap(n, pl) * 4 + 512;
}

static size_t bin_lds(const BloomPlan &pl) { return 4 * (3 * (size_t)pl.nslices + (size_t)pl.T * pl.k); }
static size_t fill_lds(const BloomPlan &pl) { return 4 * (size_t)(1u << (pl.sb - 5)); }

hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes, void *ws,
                              hipStream_t st) {
    if (bitmap_bytes == 0) return hipSuccess;
    if (n == 0 || num_probes == 0) return hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
    BloomPlan pl = bloom_plan(n, num_probes, bitmap_bytes);
    if (!ws || !plan_fits(pl, n) || fill_lds(pl) > 64 * 1024) {
        // no workspace (or a plan the binning cannot hold): device-scope atomics into the bitmap
        hipError_t e = hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
        if (e != hipSuccess) return e;
        uint64_t blocks = (n + 255) / 256;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(k_bloom_atomic, dim3((uint32_t)blocks), dim3(256), 0, st, key_bytes, key_off, n,
                           num_probes, pl.m, (uint32_t *)bitmap);
        return hipGetLastError();
    }
    static bool attrs = false;
    if (!attrs) {
        hipFuncSetAttribute((const void *)k_bloom_bin, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLds);
        hipFuncSetAttribute((const void *)k_bloom_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        (void)hipGetLastError();  // an unsupported attribute value must not poison the launch status
        attrs = true;
    }
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    BloomQueues q;
    q.cursor = (uint32_t *)w;
    q.queue = (uint32_t *)(w + cursor_bytes(pl));
    q.cap = queue_cap(n, pl);
    hipError_t e = hipMemsetAsync(q.cursor, 0, (size_t)(pl.nslices * kShards + 1) * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bloom_bin, dim3(pl.tiles), dim3(kBinThreads), bin_lds(pl), st, key_bytes, key_off, n, pl, q);
    hipLaunchKernelGGL(k_bloom_fill, dim3(pl.nslices), dim3(kFillThreads), fill_lds(pl), st, key_bytes, key_off, n, pl,
                       q, bitmap, bitmap_bytes);
    return hipGetLastError();
}

hipError_t launch_bloom_query(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes,
                              const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint8_t *result, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint32_t m = (uint32_t)(bitmap_bytes * 8);
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_bloom_query, dim3((uint32_t)blocks), dim3(256), 0, st, (const uint32_t *)bitmap,
                       num_probes, m, key_bytes, key_off, n, result);
    return hipGetLastError();
}

}  // namespace sdb
