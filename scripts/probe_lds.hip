// Probe: unaligned ds_read_b32 / ds_write_b32 on gfx950 (correctness + cycles per access).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) uint32_t lu32;
typedef __attribute__((address_space(3))) uint8_t lu8;

__global__ void k(uint32_t *out, long long *cyc, int shift, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[8192];
    for (int i = threadIdx.x; i < 8192; i += 64) buf[i] = (uint8_t)(i * 13 + 5);
    __syncthreads();
    lu8 *b = (lu8 *)buf;
    uint32_t acc = 0;
    long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        uint32_t off = (100 * threadIdx.x + shift + 4 * (it & 7)) & 4095;
        acc += *(volatile lu32 *)(b + off);
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    uint32_t off = 100 * threadIdx.x + shift;
    uint32_t v = *(volatile lu32 *)(b + off);
    uint32_t e = (uint32_t)(uint8_t)(off * 13 + 5) | ((uint32_t)(uint8_t)((off + 1) * 13 + 5) << 8) |
                 ((uint32_t)(uint8_t)((off + 2) * 13 + 5) << 16) | ((uint32_t)(uint8_t)((off + 3) * 13 + 5) << 24);
    out[64 + threadIdx.x] = (v == e);
    __syncthreads();
    long long t2 = clock64();
    for (int it = 0; it < iters; it++) {
        uint32_t o = 4096 + ((100 * threadIdx.x + shift + 4 * (it & 7)) & 2047);
        *(volatile lu32 *)(b + o) = 0x11223344u + it;
    }
    long long t3 = clock64();
    __syncthreads();
    uint32_t o = 4096 + 3000 + 16 * threadIdx.x + shift;
    *(volatile lu32 *)(b + o) = 0xA1B2C3D4u;
    __syncthreads();
    out[128 + threadIdx.x] = (b[o] == 0xD4 && b[o + 1] == 0xC3 && b[o + 2] == 0xB2 && b[o + 3] == 0xA1);
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t3 - t2;
    }
}

int main() {
    uint32_t *d;
    long long *c;
    (void)hipMalloc(&d, 4096);
    (void)hipMalloc(&c, 64);
    for (int sh = 0; sh < 4; sh++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, c, sh, 4096);
        uint32_t h[192];
        long long hc[2];
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        int okr = 1, okw = 1;
        for (int i = 0; i < 64; i++) {
            okr &= h[64 + i];
            okw &= h[128 + i];
        }
        printf("shift %d: read %s write %s | cycles/read %.1f  cycles/write %.1f\n", sh, okr ? "ok" : "BAD",
               okw ? "ok" : "BAD", hc[0] / 4096.0, hc[1] / 4096.0);
    }
    return 0;
}
