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
// Build by bucketing probes into bitmap slices, then setting bits in LDS.  Random 32-bit atomics
// to HBM/L2 run at ~25 G/s on MI355X whatever their scope (scripts/probe.hip), i.e. ~136 us for
// the 3.47 M probes of one 64 MiB SST; LDS atomics are two orders of magnitude faster.
//   k_bloom_tile  one workgroup per tile of T keys: SipHash-1-3, the k probes, an LDS counting
//                 sort by slice, and the tile's probes written slice-ordered into its own region;
//                 the per-(slice, tile) counts/offsets go to a slice-major matrix.
//   k_bloom_set   one workgroup per slice of 2^sb bits: gathers its probes from every tile region,
//                 ORs them into an LDS copy of the slice, writes the slice with plain stores.
// Deterministic (the bitmap is an OR), no global atomics, no bitmap memset.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kBloomTile = 512, kBloomTileThreads = 256;  // keys / threads per tile workgroup

__global__ __launch_bounds__(kBloomTileThreads) void k_bloom_tile(const uint8_t *__restrict__ key_bytes,
                                                    const uint64_t *__restrict__ key_off, uint64_t n,
                                                    BloomPlan pl, uint32_t *region, uint32_t *cnt,
                                                    uint32_t *off) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t *hist = lds;                                // nslices (+1)
    uint32_t *pr = lds + ((pl.nslices + 4) & ~3u);       // T * k probes
    __shared__ uint64_t s_w[17];
    const uint32_t t = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const uint64_t k0 = (uint64_t)t * pl.T;
    const uint64_t k1 = k0 + pl.T < n ? k0 + pl.T : n;
    for (uint32_t q = tid; q < pl.nslices; q += nt) hist[q] = 0;
    __syncthreads();
    for (uint64_t i = k0 + tid; i < k1; i += nt) {
        uint64_t ko = key_off[i];
        uint64_t h = siphash13(key_bytes + ko, key_off[i + 1] - ko);
        uint32_t *dst = pr + (uint32_t)(i - k0) * pl.k;
        uint32_t q = 0;
        for_each_probe(h, pl.k, pl.m, [&](uint32_t p) {
            dst[q++] = p;
            atomicAdd(&hist[p >> pl.sb], 1u);
            return true;
        });
    }
    __syncthreads();
    // exclusive scan of the slice histogram -> per-slice cursors; publish counts/offsets
    uint64_t carry = 0;
    for (uint32_t q0 = 0; q0 < pl.nslices; q0 += nt) {
        uint32_t q = q0 + tid;
        uint64_t c = q < pl.nslices ? hist[q] : 0, tot;
        uint64_t x = block_excl_scan_u64(c, s_w, &tot);
        if (q < pl.nslices) {
            cnt[(uint64_t)q * pl.tiles + t] = (uint32_t)c;
            off[(uint64_t)q * pl.tiles + t] = (uint32_t)(carry + x);
            hist[q] = (uint32_t)(carry + x);
        }
        carry += tot;
    }
    __syncthreads();
    uint32_t *reg = region + (uint64_t)t * pl.T * pl.k;
    const uint32_t np = (uint32_t)(k1 - k0) * pl.k;
    for (uint32_t q = tid; q < np; q += nt) {
        uint32_t p = pr[q];
        uint32_t pos = atomicAdd(&hist[p >> pl.sb], 1u);
        reg[pos] = p;
    }
}

__global__ __launch_bounds__(1024) void k_bloom_set(const uint32_t *__restrict__ region,
                                                    const uint32_t *__restrict__ cnt,
                                                    const uint32_t *__restrict__ off, BloomPlan pl,
                                                    uint8_t *bitmap, uint64_t bytes) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t words = 1u << (pl.sb - 5);
    uint32_t *bits = lds;                    // 2^sb bits
    uint32_t *pref = lds + words;            // tiles + 1 (exclusive scan of counts)
    uint32_t *toff = pref + pl.tiles + 4;    // tiles
    __shared__ uint64_t s_w[17];
    const uint32_t s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    for (uint32_t q = tid; q < words; q += nt) bits[q] = 0;
    uint64_t carry = 0;
    for (uint32_t t0 = 0; t0 < pl.tiles; t0 += nt) {
        uint32_t t = t0 + tid;
        uint64_t c = t < pl.tiles ? cnt[(uint64_t)s * pl.tiles + t] : 0, tot;
        uint64_t x = block_excl_scan_u64(c, s_w, &tot);
        if (t < pl.tiles) {
            pref[t] = (uint32_t)(carry + x);
            toff[t] = off[(uint64_t)s * pl.tiles + t];
        }
        carry += tot;
    }
    if (tid == 0) pref[pl.tiles] = (uint32_t)carry;
    __syncthreads();
    const uint32_t total = (uint32_t)carry;
    const uint64_t base = (uint64_t)s << pl.sb;
    const uint64_t stride = (uint64_t)pl.T * pl.k;
    for (uint32_t f = tid; f < total; f += nt) {
        // tile holding flattened probe f: last t with pref[t] <= f
        uint32_t lo = 0, hi = pl.tiles;
        while (hi - lo > 1) {
            uint32_t mid = (lo + hi) >> 1;
            if (pref[mid] <= f) lo = mid;
            else hi = mid;
        }
        uint32_t p = region[lo * stride + toff[lo] + (f - pref[lo])];
        uint32_t r = (uint32_t)(p - base);
        atomicOr(&bits[r >> 5], 1u << (r & 31));
    }
    __syncthreads();
    // slice bytes [base/8, base/8 + 2^sb/8) clipped to the bitmap
    const uint64_t b0 = base >> 3;
    const uint64_t b1 = (b0 + (words << 2)) < bytes ? b0 + (words << 2) : bytes;
    const uint64_t nfull = (b1 - b0) >> 2;
    for (uint64_t w = tid; w < nfull; w += nt) ((uint32_t *)(bitmap + b0))[w] = bits[w];
    for (uint64_t q = b0 + 4 * nfull + tid; q < b1; q += nt) {
        uint64_t r = q - b0;
        bitmap[q] = (uint8_t)(bits[r >> 2] >> (8 * (r & 3)));
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
    pl.sb = 15;  // 4 KiB slices; grow until there are at most 1024 slices
    while ((((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb) > 1024) pl.sb++;
    pl.nslices = (uint32_t)(((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb);
    if (pl.nslices == 0) pl.nslices = 1;
    // small tiles for parallelism, but at most ~4096 tiles so k_bloom_set's per-slice tile table
    // stays small; a tile's probes (T * k u32) must fit the tile kernel's LDS
    uint64_t T64 = (n + 4095) / 4096;
    if (T64 < kBloomTile) T64 = kBloomTile;
    const uint32_t tmax = 12288 / pl.k;
    uint32_t T = (uint32_t)(T64 < tmax ? T64 : tmax);
    if (T < 64) T = 64;
    pl.T = T;
    pl.tiles = (uint32_t)((n + T - 1) / T);
    if (pl.tiles == 0) pl.tiles = 1;
    return pl;
}

uint64_t bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    BloomPlan pl = bloom_plan(n, k, bitmap_bytes);
    uint64_t region = (uint64_t)pl.tiles * pl.T * pl.k * 4;
    uint64_t mat = (uint64_t)pl.tiles * pl.nslices * 4;
    return ((region + 255) & ~255ull) + 2 * ((mat + 255) & ~255ull) + 256;
}

static size_t tile_lds(const BloomPlan &pl) { return 4 * (((pl.nslices + 4) & ~3u) + (size_t)pl.T * pl.k); }
static size_t set_lds(const BloomPlan &pl) { return 4 * ((1u << (pl.sb - 5)) + 2 * (size_t)pl.tiles + 8); }

hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes, void *ws,
                              hipStream_t st) {
    if (bitmap_bytes == 0) return hipSuccess;
    if (n == 0 || num_probes == 0) return hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
    BloomPlan pl = bloom_plan(n, num_probes, bitmap_bytes);
    if (!ws || tile_lds(pl) > 96 * 1024 || set_lds(pl) > 128 * 1024) {
        // no workspace (or a plan that does not fit LDS): device-scope atomics into the bitmap
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
        hipFuncSetAttribute((const void *)k_bloom_tile, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        hipFuncSetAttribute((const void *)k_bloom_set, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
        attrs = true;
    }
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    uint64_t region_b = (((uint64_t)pl.tiles * pl.T * pl.k * 4) + 255) & ~255ull;
    uint64_t mat_b = (((uint64_t)pl.tiles * pl.nslices * 4) + 255) & ~255ull;
    uint32_t *region = (uint32_t *)w, *cnt = (uint32_t *)(w + region_b), *off = (uint32_t *)(w + region_b + mat_b);
    hipLaunchKernelGGL(k_bloom_tile, dim3(pl.tiles), dim3(kBloomTileThreads), tile_lds(pl), st, key_bytes, key_off, n, pl, region,
                       cnt, off);
    hipLaunchKernelGGL(k_bloom_set, dim3(pl.nslices), dim3(1024), set_lds(pl), st, region, cnt, off, pl, bitmap,
                       bitmap_bytes);
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
