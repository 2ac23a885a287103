// tools/ubench_sha1.hip -- throughput of the generated SHA-1 compression (no memory traffic) at
// 1/2/4/8 waves per SIMD: separates the VALU-mix / issue limit from memory and clock effects.
// Build: hipcc --offload-arch=gfx950 -O3 -I torrent_amd/csrc tools/ubench_sha1.hip -o tools/ubench_sha1_bin
// "SIMD cycles per compression" (event time x clock / compressions per SIMD) is the number to read;
// 8 waves per SIMD = two 1024-thread blocks per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "sha1_asm.h"

__global__ __launch_bounds__(1024) void kfull(uint32_t* out, int iters, uint64_t* clk) {
    uint32_t h[5] = {threadIdx.x, 2, 3, 4, 5};
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * (i + 1);
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        uint32_t r[5];
        tv_sha1_full(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ w[3];
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

// two compressions per loop trip (the lane kernel's unroll): halves the loop's SALU + branch share
__global__ __launch_bounds__(1024) void kfull2(uint32_t* out, int iters, uint64_t* clk) {
    uint32_t h[5] = {threadIdx.x, 2, 3, 4, 5};
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * (i + 1);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it += 2) {
        uint32_t r[5];
        tv_sha1_full(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
        tv_sha1_full(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ w[3];
    if (threadIdx.x == 0) clk[2 * blockIdx.x] = t1 - t0;
}

int main() {
    uint32_t* out; uint64_t* clk;
    hipMalloc(&out, 4 << 22); hipMalloc(&clk, 8 * 4096);
    const int iters = 2000;
    for (int wps : {1, 2, 4, 8}) {
        const int threads = 64 * 4 * (wps > 4 ? 4 : wps);  // wps waves on each of the 4 SIMDs
        const int blocks = 256 * (wps > 4 ? wps / 4 : 1);
        hipLaunchKernelGGL(kfull, dim3(blocks), dim3(threads), 0, 0, out, 50, clk);
        hipDeviceSynchronize();
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kfull, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;  // memtime cycles / realtime(100 MHz)
        const double lanes = (double)blocks * threads;
        const double gbps = lanes * iters * 64.0 / (ms / 1e3) / 1e9;
        const double instr_per_simd = (double)iters * 597 * wps;
        printf("  SIMD cycles per compression (event time x clock): %.0f\n", ms * 1e-3 * ghz * 1e9 / (iters * (double)wps));  // ~597 VALU per compression incl. feed-forward
        printf("waves/SIMD=%d  %.3f ms  clock %.2f GHz  %.1f GB/s-equiv  %.2f cycles/VALU per SIMD  %.2f cycles/VALU per wave\n",
               wps, ms, ghz, gbps, (double)c[0] / instr_per_simd, (double)c[0] / (iters * 597.0));
    }
    // Lone-wave cadence against CU occupancy: 1, 2, 4 waves per CU (one per SIMD, 256 blocks), cycles
    // per compression from block 0's own s_memtime span (core clock), so no clock estimate enters.
    for (int threads : {64, 128, 256}) {
        hipLaunchKernelGGL(kfull, dim3(256), dim3(threads), 0, 0, out, 50, clk);
        hipLaunchKernelGGL(kfull, dim3(256), dim3(threads), 0, 0, out, iters, clk);
        hipDeviceSynchronize();
        uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        printf("waves/CU=%d (1 per SIMD used)  block-0 memtime cycles per compression %.0f  (%.3f per VALU of ~597)\n",
               threads / 64, (double)c[0] / iters, (double)c[0] / iters / 597.0);
    }
    {
        hipLaunchKernelGGL(kfull2, dim3(256), dim3(64), 0, 0, out, 50, clk);
        hipLaunchKernelGGL(kfull2, dim3(256), dim3(64), 0, 0, out, iters, clk);
        hipDeviceSynchronize();
        uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        printf("2 compressions per trip, waves/CU=1  block-0 memtime cycles per compression %.0f  (%.3f per VALU of ~597)\n",
               (double)c[0] / iters, (double)c[0] / iters / 597.0);
    }
    return 0;
}
