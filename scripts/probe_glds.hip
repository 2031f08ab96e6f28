// Probe: LDS-DMA (global_load_lds_dword) from byte-unaligned global addresses on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__global__ void k(const uint8_t *src, uint8_t *out, int shift) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = 0xdeadbeef;
    __syncthreads();
    uint32_t base = (uint32_t)(uintptr_t)(lds_void *)buf;
    // lanes 0..39 active, dest dwords 8.. (LDS byte base + 32)
    if (threadIdx.x < 40)
        __builtin_amdgcn_global_load_lds((glb_void *)(src + shift + 4 * threadIdx.x), (lds_void *)(uintptr_t)(base + 32), 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) ((uint32_t *)out)[i] = buf[i];
}

int main() {
    uint8_t h[4096], o[4096];
    for (int i = 0; i < 4096; i++) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *d, *dout;
    hipMalloc(&d, 4096);
    hipMalloc(&dout, 4096);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    int bad = 0;
    for (int sh = 0; sh < 8; sh++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, dout, sh);
        hipMemcpy(o, dout, 4096, hipMemcpyDeviceToHost);
        int ok = 1;
        for (int i = 0; i < 160; i++) if (o[32 + i] != h[sh + i]) ok = 0;
        uint32_t w7 = ((uint32_t *)o)[7], w48 = ((uint32_t *)o)[48];
        printf("shift %d: %s (guard %08x %08x)\n", sh, ok ? "ok" : "MISMATCH", w7, w48);
        if (!ok) { bad = 1; for (int i = 0; i < 12; i++) printf("%02x/%02x ", o[32 + i], h[sh + i]); printf("\n"); }
    }
    return bad;
}
