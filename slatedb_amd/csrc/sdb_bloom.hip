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

__global__ __launch_bounds__(256) void k_bloom_build(const uint8_t *__restrict__ key_bytes,
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

hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes,
                              hipStream_t st) {
    hipError_t e = hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
    if (e != hipSuccess || bitmap_bytes == 0 || n == 0 || num_probes == 0) return e;
    uint32_t m = (uint32_t)(bitmap_bytes * 8);
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_bloom_build, dim3((uint32_t)blocks), dim3(256), 0, st, key_bytes, key_off, n,
                       num_probes, m, (uint32_t *)bitmap);
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
