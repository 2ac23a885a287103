// simd_probe.hip -- where does a 512-thread, 160 KiB-LDS workgroup put its 8 waves?  (the duo kernel's
// premise: waves w and w + 4 share SIMD w % 4, and one such workgroup runs per CU).
//
//   hipcc --offload-arch=gfx950 -O2 -o build/simd_probe tools/simd_probe.hip && build/simd_probe
//
// Each wave records HW_REG_HW_ID (wave [3:0], simd [5:4], cu [11:8], sh [12], se [15:13]) and
// HW_REG_XCC_ID, then spins ~200 us so every workgroup of the grid is resident at once.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <set>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(512) void probe(uint32_t* out, int lds_bytes_used) {
    __shared__ uint32_t lds[160 * 1024 / 4];
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    lds[threadIdx.x] = hw;                       // keep the array alive
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 20000) __builtin_amdgcn_s_sleep(4);   // 200 us at 100 MHz
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = threadIdx.x >> 6;
        out[(blockIdx.x * 8 + w) * 2 + 0] = lds[(threadIdx.x + 64 * lds_bytes_used) & 511];
        out[(blockIdx.x * 8 + w) * 2 + 1] = xcc;
    }
}

int main() {
    for (int grid : {200, 256}) {
        uint32_t* d;
        if (hipMalloc(&d, grid * 8 * 2 * 4) != hipSuccess) return 1;
        hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, d, 0);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        std::vector<uint32_t> h(grid * 16);
        hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
        hipFree(d);
        int paired = 0, bad = 0;
        std::set<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>> cus;
        for (int b = 0; b < grid; b++) {
            uint32_t simd[8];
            for (int w = 0; w < 8; w++) simd[w] = (h[(b * 8 + w) * 2] >> 4) & 3;
            const uint32_t hw0 = h[b * 16], xcc = h[b * 16 + 1] & 0xF;
            cus.insert({xcc, (hw0 >> 13) & 7, (hw0 >> 12) & 1, (hw0 >> 8) & 15});
            bool ok = true;
            for (int w = 0; w < 4; w++) ok &= simd[w] == simd[w + 4];
            std::set<uint32_t> first(simd, simd + 4);
            ok &= first.size() == 4;
            paired += ok;
            if (!ok && bad++ < 8) {
                printf("grid %d wg %d simd of waves 0..7:", grid, b);
                for (int w = 0; w < 8; w++) printf(" %u", simd[w]);
                printf("\n");
            }
            if (b < 4) {
                printf("grid %d wg %d xcc %u hw_id %08x simd of waves 0..7:", grid, b, xcc, hw0);
                for (int w = 0; w < 8; w++) printf(" %u", simd[w]);
                printf("\n");
            }
        }
        printf("grid %d: %d of %d workgroups have waves w, w+4 on one SIMD and waves 0-3 on 4 SIMDs; %zu distinct CUs\n",
               grid, paired, grid, cus.size());
    }
    return 0;
}
