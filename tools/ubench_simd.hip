// tools/ubench_simd.hip -- SIMD-level VALU throughput on gfx950 for the SHA-1 instruction kinds.
//
// Question: how many cycles does one SIMD spend per wave64 integer instruction when several waves
// share it?  (MI355X_MICROARCH.md: v_fma_f32 runs at 2 cyc per wave64 on the 32-lane SIMD; a lone
// wave issues every ~4.)  If integer VOP3 ops also took 2 cycles, the SHA-1 VALU roofline would be
// 2x the 4.1 TB/s DESIGN.md uses.
//
// Each wave runs 8 independent chains of one instruction kind for ITERS x 64 instructions (no
// memory traffic).  Grid: 256 x B workgroups of 256 threads (4 waves per CU per workgroup, one per
// SIMD); B = waves per SIMD.  Time = HIP events around the launch; the shader clock is measured
// with s_memtime on each wave (cycles) vs the event time.  Output: SIMD cycles per wave64
// instruction = (event time x clock) / (wave-instructions per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_simd.hip -o tools/ubench_simd
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define REP8(x) x x x x x x x x
#define CHAINS8(op) \
    asm volatile(REP8(op(%0) op(%1) op(%2) op(%3) op(%4) op(%5) op(%6) op(%7)) \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(k1), "v"(k2))

#define OP_ADD(r) "v_add_u32 " #r ", " #r ", %8\n"
#define OP_XOR(r) "v_xor_b32 " #r ", " #r ", %8\n"
#define OP_ADD3(r) "v_add3_u32 " #r ", " #r ", %8, %9\n"
#define OP_ALIGN(r) "v_alignbit_b32 " #r ", " #r ", " #r ", 27\n"
#define OP_BITOP3(r) "v_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x96\n"
#define OP_FMA(r) "v_fma_f32 " #r ", " #r ", %8, %9\n"
#define OP_BFI(r) "v_bfi_b32 " #r ", " #r ", %8, %9\n"
#define OP_PERM(r) "v_perm_b32 " #r ", 0, " #r ", %8\n"
#define OP_LSHLOR(r) "v_lshl_or_b32 " #r ", " #r ", 5, %8\n"
#define OP_LSHLADD(r) "v_lshl_add_u32 " #r ", " #r ", 5, %8\n"
#define OP_ADDE64(r) "v_add_u32_e64 " #r ", " #r ", %8\n"

constexpr int ITERS = 1024;  // x 64 instructions per wave

template <int T>
__global__ __launch_bounds__(256) void kbench(uint64_t* cyc, uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u, g = a * 17u,
             h = a * 19u, k1 = seed | 1u, k2 = seed * 7u;
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int it = 0; it < ITERS; it++) {
        if constexpr (T == 0) CHAINS8(OP_ADD);
        else if constexpr (T == 1) CHAINS8(OP_XOR);
        else if constexpr (T == 2) CHAINS8(OP_ADD3);
        else if constexpr (T == 3) CHAINS8(OP_ALIGN);
        else if constexpr (T == 4) CHAINS8(OP_BITOP3);
        else if constexpr (T == 5) CHAINS8(OP_FMA);
        else if constexpr (T == 6) CHAINS8(OP_BFI);
        else if constexpr (T == 7) CHAINS8(OP_PERM);
        else if constexpr (T == 8) CHAINS8(OP_LSHLOR);
        else if constexpr (T == 9) CHAINS8(OP_LSHLADD);
        else CHAINS8(OP_ADDE64);
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

static const char* kNames[] = {"v_add_u32 (VOP2)", "v_xor_b32 (VOP2)", "v_add3_u32", "v_alignbit_b32",
                               "v_bitop3_b32", "v_fma_f32 (control)", "v_bfi_b32", "v_perm_b32",
                               "v_lshl_or_b32", "v_lshl_add_u32", "v_add_u32_e64 (VOP3)"};

template <int T>
static void run(int per_simd) {
    const int blocks = 256 * per_simd;
    uint64_t* cyc;
    uint32_t* sink;
    (void)hipMalloc(&cyc, blocks * 4 * sizeof(uint64_t));
    (void)hipMalloc(&sink, blocks * 256 * sizeof(uint32_t));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kbench<T>, dim3(blocks), dim3(256), 0, 0, cyc, sink, 12345u);  // warm up
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kbench<T>, dim3(blocks), dim3(256), 0, 0, cyc, sink, 777u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(blocks * 4);
    (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    uint64_t mx = 0;
    double sum = 0;
    for (uint64_t v : h) {
        mx = v > mx ? v : mx;
        sum += (double)v;
    }
    const double instr_per_wave = (double)ITERS * 64;
    // clock from the longest wave's s_memtime span over the event time (an upper bound on the span)
    const double clk_ghz = (double)mx / (ms * 1e6);
    const double simd_cyc = (ms * 1e6 * clk_ghz) / (instr_per_wave * per_simd);
    const double wave_cyc = (sum / h.size()) / instr_per_wave;
    printf("%-20s waves/SIMD=%d : %.3f ms, clock ~%.2f GHz, SIMD %.2f cyc per wave64 instr, "
           "one wave %.2f cyc/instr\n",
           kNames[T], per_simd, ms, clk_ghz, simd_cyc, wave_cyc);
    (void)hipFree(cyc);
    (void)hipFree(sink);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<0>(w);
        run<1>(w);
        run<2>(w);
        run<3>(w);
        run<4>(w);
        run<5>(w);
        run<6>(w);
        run<7>(w);
        run<8>(w);
        run<9>(w);
        run<10>(w);
    }
    return 0;
}
