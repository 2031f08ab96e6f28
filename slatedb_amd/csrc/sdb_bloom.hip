// sdb_bloom.hip — bloom filter build / probe for gfx950.
//
// Replaces BloomFilterBuilder (slatedb/src/filter.rs:40-90) and BloomFilter::might_contain
// (filter.rs:124-136): filter_hash = SipHash-1-3 with a zero key over the raw key bytes
// (siphasher 1.0.3, filter.rs:196-204); probes by enhanced double hashing (filter.rs:206-221);
// LSB-first bit order (filter.rs:223-233).  Bit p of the byte-addressed bitmap is bit (p & 31) of the
// little-endian 32-bit word p >> 5, so setting it is one 32-bit atomicOr.
#include <mutex>

#include "sdb_bloom.h"

namespace sdb {

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

__global__ __launch_bounds__(kBinThreads) void k_bloom_bin(const uint8_t *__restrict__ key_bytes,
                                                           const uint64_t *__restrict__ key_off, uint64_t n,
                                                           BloomPlan pl, BloomSlots q) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    bloom_bin_tile(blockIdx.x, key_bytes, key_off, n, pl, q, lds);
}

__global__ __launch_bounds__(kFillThreads) void k_bloom_fill(const uint8_t *__restrict__ key_bytes,
                                                             const uint64_t *__restrict__ key_off, uint64_t n,
                                                             BloomPlan pl, BloomSlots q, uint8_t *bitmap,
                                                             uint64_t bytes) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    bloom_fill_slice(blockIdx.x, key_bytes, key_off, n, pl, q, bitmap, bytes, lds);
}

// Byte-granular probe reads: the bitmap may sit at any address (e.g. 17 bytes into an SST's filter
// block, format/sst.rs:394-421) and is read only inside [0, ceil(m / 8)).
__global__ __launch_bounds__(256) void k_bloom_query(const uint8_t *bitmap, uint32_t k, uint32_t m,
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
                if (!((bitmap[p >> 3] >> (p & 7)) & 1u)) {
                    r = 0;
                    return false;
                }
                return true;
            });
        }
        result[i] = r;
    }
}

BloomPlan bloom_plan(uint64_t n, uint32_t k, uint64_t bitmap_bytes, uint32_t tile_keys) {
    BloomPlan pl{};
    pl.k = k ? k : 1;
    pl.m = (uint32_t)(bitmap_bytes * 8);
    // slices of 2^sb bits: at least 4 KiB, at most 64 KiB of LDS, and at most 256 of them
    pl.sb = 15;
    while (pl.sb < 19 && (((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb) > 256) pl.sb++;
    pl.nslices = (uint32_t)(((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb);
    if (pl.nslices == 0) pl.nslices = 1;
    uint32_t T = tile_keys;
    if (!T) {  // kBinKeysPerThread keys per thread, fewer when the sorted probes outgrow LDS
        T = kBinThreads * kBinKeysPerThread;
        while (T > kBinThreads && 4ull * (2 * pl.nslices + (uint64_t)T * pl.k) > kBinLds) T -= kBinThreads;
    }
    pl.T = T;
    pl.tiles = (uint32_t)((n + T - 1) / T);
    if (pl.tiles == 0) pl.tiles = 1;
    pl.mmod = pl.m ? ~0ull / pl.m + 1 : 0;
    return pl;
}

uint32_t bloom_slot_cap(const BloomPlan &pl) {
    // uniform probes: a slot (slice, tile) receives the probes of the tile's T keys that land in the
    // slice (2^sb of the m bits); + 6 sigma + 16
    const double frac = pl.m ? (double)(1ull << pl.sb) / pl.m : 1.0;
    const double mean = (double)pl.T * pl.k * (frac < 1.0 ? frac : 1.0);
    uint64_t cap = (uint64_t)(mean + 6.0 * __builtin_sqrt(mean + 1.0)) + 16;
    cap = (cap + 3) & ~3ull;
    const uint64_t most = (uint64_t)pl.T * pl.k;  // a slot never holds more than the tile's probes
    if (cap > most) cap = (most + 3) & ~3ull;
    return (uint32_t)cap;
}

bool bloom_plan_fits(const BloomPlan &pl) {
    return pl.k <= kBinMaxK && pl.sb <= 19 && pl.m >= 2 && bloom_bin_lds(pl) <= kBinLds &&
           bloom_fill_lds(pl) <= 96 * 1024;
}

uint64_t bloom_slots_bytes(const BloomPlan &pl) {
    const uint64_t counts = ((uint64_t)pl.tiles * pl.nslices * 4 + 255) & ~255ull;
    return 256 + counts + (uint64_t)pl.nslices * pl.tiles * bloom_slot_cap(pl) * 4;
}

uint64_t bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    return bloom_slots_bytes(bloom_plan(n, k, bitmap_bytes));
}

BloomSlots bloom_slots(void *ws, const BloomPlan &pl) {
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    BloomSlots q;
    q.count = (uint32_t *)w;
    q.slot = (uint32_t *)(w + (((uint64_t)pl.tiles * pl.nslices * 4 + 255) & ~255ull));
    q.cap = bloom_slot_cap(pl);
    return q;
}

size_t bloom_bin_lds(const BloomPlan &pl) { return 4 * (2 * (size_t)pl.nslices + (size_t)pl.T * pl.k); }
size_t bloom_fill_lds(const BloomPlan &pl) { return 4 * ((size_t)(1u << (pl.sb - 5)) + pl.tiles); }

hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes, void *ws,
                              hipStream_t st) {
    if (bitmap_bytes == 0) return hipSuccess;
    if (n == 0 || num_probes == 0) return hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
    BloomPlan pl = bloom_plan(n, num_probes, bitmap_bytes);
    if (!ws || !bloom_plan_fits(pl)) {
        // no workspace (or a plan the binning cannot hold): device-scope atomics into the bitmap
        hipError_t e = hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
        if (e != hipSuccess) return e;
        uint64_t blocks = (n + 255) / 256;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(k_bloom_atomic, dim3((uint32_t)blocks), dim3(256), 0, st, key_bytes, key_off, n,
                           num_probes, pl.m, (uint32_t *)bitmap);
        return hipGetLastError();
    }
    static std::once_flag attrs;
    std::call_once(attrs, [] {
        (void)hipFuncSetAttribute((const void *)k_bloom_bin, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLds);
        (void)hipFuncSetAttribute((const void *)k_bloom_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        (void)hipGetLastError();  // an unsupported attribute value must not poison the launch status
    });
    const BloomSlots q = bloom_slots(ws, pl);
    hipLaunchKernelGGL(k_bloom_bin, dim3(pl.tiles), dim3(kBinThreads), bloom_bin_lds(pl), st, key_bytes, key_off, n, pl, q);
    hipLaunchKernelGGL(k_bloom_fill, dim3(pl.nslices), dim3(kFillThreads), bloom_fill_lds(pl), st, key_bytes, key_off, n, pl,
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
    hipLaunchKernelGGL(k_bloom_query, dim3((uint32_t)blocks), dim3(256), 0, st, bitmap,
                       num_probes, m, key_bytes, key_off, n, result);
    return hipGetLastError();
}

}  // namespace sdb

namespace sdb {
// The encode workspace serves either build: the fused one (tiles = k_seg's chunks) or the standalone
// kernels (sdb_encode_sst falls back to them when the fused plan does not fit).
uint64_t encode_bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    const uint64_t a = bloom_workspace_bytes(n, k, bitmap_bytes);
    const uint64_t b = bloom_slots_bytes(bloom_plan(n, k, bitmap_bytes, kChunk));
    return a > b ? a : b;
}
}  // namespace sdb
