// tools/ubench_lanes.hip -- does a wave with fewer active lanes issue the SHA-1 block faster?
// One wave per SIMD (4 per CU), ACTIVE lanes per wave executing tv_sha1_full in a loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "sha1_asm.h"

__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, int active) {
    if ((int)(threadIdx.x & 63) >= active) return;
    uint32_t h[5] = {threadIdx.x, 2, 3, 4, 5};
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * (i + 1);
    for (int it = 0; it < iters; it++) {
        uint32_t r[5];
        tv_sha1_full(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ w[3];
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 4 << 22);
    const int iters = 2000;
    for (int wps : {1, 2})
        for (int active : {64, 32, 16, 8}) {
            hipLaunchKernelGGL(k, dim3(256 * wps), dim3(256), 0, 0, out, 50, active);
            (void)hipDeviceSynchronize();
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(256 * wps), dim3(256), 0, 0, out, iters, active);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            const double cyc = ms * 1e-3 * 2.4e9 / (iters * 597.0) ;  // per wave-instruction at 2.4 GHz
            printf("waves/SIMD=%d active lanes=%2d  %.3f ms  %.2f cycles/VALU(@2.4GHz) per wave  piece-rate %.1f MB/s/lane\n",
                   wps, active, ms, cyc, iters * 64.0 / (ms * 1e-3) / 1e6);
        }
    return 0;
}
