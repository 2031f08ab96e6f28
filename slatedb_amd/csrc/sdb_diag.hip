// sdb_diag.hip — diagnostic entry points that pin device primitives on their own: the matrix-core wave
// CRC against the slicing-by-8 one (and, in the tests, Python's zlib.crc32), and the i8 MFMA lane maps.
#include "sdb_crc_mfma.h"

namespace sdb {

__global__ __launch_bounds__(64) void k_diag_mfma_i8(const int32_t *a, const int32_t *b, int32_t *d) {
    const uint32_t l = threadIdx.x;
    const i32x4 av = {a[4 * l], a[4 * l + 1], a[4 * l + 2], a[4 * l + 3]};
    const i32x4 bv = {b[4 * l], b[4 * l + 1], b[4 * l + 2], b[4 * l + 3]};
    i32x16 acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
    for (int i = 0; i < 16; i++) d[16 * l + i] = acc[i];
}

constexpr uint32_t kDiagWaves = 4, kDiagWaveLds = 64 + 4096 + 64;

// one wave per range: stage it after a 64-byte zero guard (16-byte granules), invert bytes [0, 4)
// (crc32fast's init), then the wave CRC
template <int METHOD>
__global__ __launch_bounds__(64 * kDiagWaves) void k_diag_crc(const uint8_t *data, const uint64_t *off, uint64_t n,
                                                              uint32_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (lds_addr((const void *)smem) != 0) return;
    const uint32_t tab = METHOD ? kCrcMfmaLds : kCrcTablesLds;
    if (METHOD) crc_mfma_tables_to_lds((lu32 *)smem);
    else crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    lu8 *img = (lu8 *)smem + tab + w * kDiagWaveLds + 64;
    for (uint64_t i = (uint64_t)blockIdx.x * kDiagWaves + w; i < n; i += (uint64_t)gridDim.x * kDiagWaves) {
        const uint64_t s = off[i], e = off[i + 1];
        const uint32_t L = (uint32_t)(e - s);
        if (l < 16) ((lu32 *)(img - 64))[l] = 0;
        for (uint32_t q = l; q < (L + 63) / 64 * 64 + 64; q += 64) img[q] = q < L ? data[s + q] : 0;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (l < 4) img[l] = (uint8_t)~img[l];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t c = METHOD ? wave_crc_image_mfma<>(img, L) : wave_crc_image_ra(img, L);
        if (l == 0) out[i] = c;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// STREAM-like copy: 16 bytes per lane, four loads in flight per lane before their stores, grid-stride
// (the attainable HBM ceiling the roofline fractions are compared with, beside the 8 TB/s spec)
__global__ __launch_bounds__(256) void k_diag_copy(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
        const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride), d = __builtin_nontemporal_load(src + i + 3 * stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
        __builtin_nontemporal_store(c, dst + i + 2 * stride);
        __builtin_nontemporal_store(d, dst + i + 3 * stride);
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

// Copy-ceiling probes (mode): 1 plain loads / stores in the grid-stride pattern of k_diag_copy; 2 each wave
// copies 4 KiB contiguous per step (4 x 16 B per lane, loads before stores); 3 read only (a xor-reduction
// per thread, stored once); 4 write only.
template <int MODE>
__global__ __launch_bounds__(256) void k_diag_bw(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (MODE == 1) {
        uint64_t i = t;
        for (; i + 3 * stride < n16; i += 4 * stride) {
            const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
            dst[i] = a;
            dst[i + stride] = b;
            dst[i + 2 * stride] = c;
            dst[i + 3 * stride] = d;
        }
        for (; i < n16; i += stride) dst[i] = src[i];
    } else if (MODE == 2) {
        const uint64_t w = t >> 6, nw = stride >> 6, l = t & 63;
        for (uint64_t b = w * 256; b + 256 <= n16; b += nw * 256) {
            const u32x4 a = src[b + l], c = src[b + 64 + l], d = src[b + 128 + l], e = src[b + 192 + l];
            dst[b + l] = a;
            dst[b + 64 + l] = c;
            dst[b + 128 + l] = d;
            dst[b + 192 + l] = e;
        }
    } else if (MODE == 3) {
        u32x4 x = {0, 0, 0, 0};
        uint64_t i = t;
        for (; i + 3 * stride < n16; i += 4 * stride) {
            const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
            x ^= a ^ b ^ c ^ d;
        }
        for (; i < n16; i += stride) x ^= src[i];
        if (t < n16) dst[t] = x;
    } else {
        const u32x4 v = {(uint32_t)t, 1u, 2u, 3u};
        for (uint64_t i = t; i < n16; i += stride) dst[i] = v;
    }
}

}  // namespace sdb

using namespace sdb;

extern "C" sdb_status sdb_diag_bw(void *dst, const void *src, uint64_t bytes, int mode, int wg_per_cu, void *stream) {
    if (!dst || !src || (bytes & 4095) || (((uintptr_t)dst | (uintptr_t)src) & 15) || mode < 0 || mode > 4 || wg_per_cu < 1)
        return SDB_INVALID_ARGUMENT;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const dim3 g((uint32_t)(wg_per_cu * cus)), b(256);
    hipStream_t st = (hipStream_t)stream;
    u32x4 *d = (u32x4 *)dst;
    const u32x4 *s = (const u32x4 *)src;
    const uint64_t n = bytes / 16;
    switch (mode) {
        case 0: hipLaunchKernelGGL(k_diag_copy, g, b, 0, st, d, s, n); break;
        case 1: hipLaunchKernelGGL(k_diag_bw<1>, g, b, 0, st, d, s, n); break;
        case 2: hipLaunchKernelGGL(k_diag_bw<2>, g, b, 0, st, d, s, n); break;
        case 3: hipLaunchKernelGGL(k_diag_bw<3>, g, b, 0, st, d, s, n); break;
        default: hipLaunchKernelGGL(k_diag_bw<4>, g, b, 0, st, d, s, n); break;
    }
    return hipGetLastError() == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;
}

extern "C" sdb_status sdb_diag_copy(void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!dst || !src || (bytes & 15) || (((uintptr_t)dst | (uintptr_t)src) & 15)) return SDB_INVALID_ARGUMENT;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipLaunchKernelGGL(k_diag_copy, dim3(8 * cus), dim3(256), 0, (hipStream_t)stream, (u32x4 *)dst, (const u32x4 *)src,
                       bytes / 16);
    return hipGetLastError() == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;
}

extern "C" sdb_status sdb_diag_mfma_i8(const int32_t *a, const int32_t *b, int32_t *d, void *stream) {
    if (!a || !b || !d) return SDB_INVALID_ARGUMENT;
    hipLaunchKernelGGL(k_diag_mfma_i8, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, d);
    return hipGetLastError() == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;
}

extern "C" sdb_status sdb_diag_crc32_blocks(const uint8_t *data, const uint64_t *off, uint64_t n, uint32_t *out,
                                            int method, void *stream) {
    if (!n) return SDB_OK;
    if (!data || !off || !out || method < 0 || method > 1) return SDB_INVALID_ARGUMENT;
    const uint32_t lds = (method ? kCrcMfmaLds : kCrcTablesLds) + kDiagWaves * kDiagWaveLds;
    const uint32_t grid = (uint32_t)((n + kDiagWaves - 1) / kDiagWaves < 1024 ? (n + kDiagWaves - 1) / kDiagWaves : 1024);
    if (method) {
        (void)hipFuncSetAttribute((const void *)k_diag_crc<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_diag_crc<1>, dim3(grid), dim3(64 * kDiagWaves), lds, (hipStream_t)stream, data, off, n, out);
    } else {
        (void)hipFuncSetAttribute((const void *)k_diag_crc<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_diag_crc<0>, dim3(grid), dim3(64 * kDiagWaves), lds, (hipStream_t)stream, data, off, n, out);
    }
    return hipGetLastError() == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;
}
