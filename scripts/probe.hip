// probe.hip — microbenchmarks that inform the bloom design (not product code):
//   1. which XCD (HW_REG_XCC_ID) each workgroup runs on
//   2. random 32-bit atomicOr throughput: device scope vs workgroup scope into per-XCD replicas
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__device__ uint32_t xcc() { return (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | ((4 - 1) << 11)); }

__global__ void k_xcc(uint32_t *out) { if (threadIdx.x == 0) out[blockIdx.x] = xcc(); }

__device__ uint32_t mix(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }

template <int MODE>
__global__ void k_atom(uint32_t *bm, uint32_t words, uint32_t n, uint64_t rw) {
    uint32_t *dst = bm;
    if (MODE == 1) dst = bm + (uint64_t)(xcc() & 7) * rw;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t h = mix(i * 2654435761u + 12345);
        uint32_t w = h % words;
        if (MODE == 0) atomicOr(dst + w, 1u << (h & 31));
        else if (MODE == 1) __hip_atomic_fetch_or(dst + w, 1u << (h & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_fetch_or(dst + w, 1u << (h & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 4096 * 4);
    hipLaunchKernelGGL(k_xcc, dim3(4096), dim3(64), 0, 0, d);
    std::vector<uint32_t> h(4096);
    hipMemcpy(h.data(), d, 4096 * 4, hipMemcpyDeviceToHost);
    int cnt[16] = {0};
    for (int i = 0; i < 4096; i++) cnt[h[i] & 15]++;
    printf("xcc ids (first 16 blocks):");
    for (int i = 0; i < 16; i++) printf(" %u", h[i]);
    printf("\nxcc histogram:");
    for (int i = 0; i < 16; i++) printf(" %d", cnt[i]);
    printf("\n");
    // atomics: 3.47M random bits into a 723 KB bitmap (D1 bloom shape)
    uint32_t words = 723155 / 4 + 1, n = 3471144;
    uint64_t rw = (words + 63) & ~63u;
    uint32_t *bm;
    hipMalloc(&bm, rw * 4 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[3] = {"device-scope atomicOr (1 bitmap)", "workgroup-scope into per-XCD replicas", "agent-scope __hip_atomic"};
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            hipMemset(bm, 0, rw * 4 * 8);
            hipEventRecord(a, 0);
            if (mode == 0) hipLaunchKernelGGL(k_atom<0>, dim3(2048), dim3(256), 0, 0, bm, words, n, rw);
            if (mode == 1) hipLaunchKernelGGL(k_atom<1>, dim3(2048), dim3(256), 0, 0, bm, words, n, rw);
            if (mode == 2) hipLaunchKernelGGL(k_atom<2>, dim3(2048), dim3(256), 0, 0, bm, words, n, rw);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("%-45s %8.1f us  (%.1f G atomics/s)\n", names[mode], ms * 1e3, n / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
