// tools/ubench_valu.hip -- gfx950 VALU latency / issue microbenchmark for the SHA-1 round ops.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
// Each test runs an asm block of REPS x BODY instructions and reports shader cycles per
// instruction (s_memtime), for 1 wave per CU and for W waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int T>
__global__ void kbench(uint64_t* cyc, uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u, g = a * 17u, h = a * 19u;
    uint64_t t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int it = 0; it < 16; it++) {
        if constexpr (T == 0) {  // dependent v_add3_u32 chain
            asm volatile(REP64("v_add3_u32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c));
        } else if constexpr (T == 1) {  // dependent v_alignbit chain
            asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 27\n") : "+v"(a));
        } else if constexpr (T == 2) {  // dependent v_add_u32 (VOP2) chain
            asm volatile(REP64("v_add_u32 %0, %0, %1\n") : "+v"(a) : "v"(b));
        } else if constexpr (T == 3) {  // dependent v_bitop3 chain
            asm volatile(REP64("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n") : "+v"(a) : "v"(b), "v"(c));
        } else if constexpr (T == 4) {  // alternating alignbit -> add3 (the SHA-1 round critical path)
            asm volatile(REP64("v_alignbit_b32 %1, %0, %0, 27\n v_add3_u32 %0, %1, %2, %3\n") : "+v"(a), "+v"(b) : "v"(c), "v"(d));
        } else if constexpr (T == 5) {  // 4 independent add3 chains interleaved (issue rate)
            asm volatile(REP64("v_add3_u32 %0, %0, %4, %5\n v_add3_u32 %1, %1, %4, %5\n v_add3_u32 %2, %2, %4, %5\n v_add3_u32 %3, %3, %4, %5\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
        } else if constexpr (T == 6) {  // 8 independent alignbit
            asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 27\n v_alignbit_b32 %1, %1, %1, 27\n v_alignbit_b32 %2, %2, %2, 27\n v_alignbit_b32 %3, %3, %3, 27\n"
                               "v_alignbit_b32 %4, %4, %4, 27\n v_alignbit_b32 %5, %5, %5, 27\n v_alignbit_b32 %6, %6, %6, 27\n v_alignbit_b32 %7, %7, %7, 27\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
        } else if constexpr (T == 7) {  // 8 independent bitop3
            asm volatile(REP64("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n v_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n v_bitop3_b32 %2, %2, %3, %4 bitop3:0x96\n v_bitop3_b32 %3, %3, %4, %5 bitop3:0x96\n"
                               "v_bitop3_b32 %4, %4, %5, %6 bitop3:0x96\n v_bitop3_b32 %5, %5, %6, %7 bitop3:0x96\n v_bitop3_b32 %6, %6, %7, %0 bitop3:0x96\n v_bitop3_b32 %7, %7, %0, %1 bitop3:0x96\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
        } else if constexpr (T == 8) {  // dependent chain with 1 independent op between links
            asm volatile(REP64("v_add3_u32 %0, %0, %2, %3\n v_add3_u32 %1, %1, %2, %3\n") : "+v"(a), "+v"(b) : "v"(c), "v"(d));
        } else if constexpr (T == 9) {  // dependent v_lshl_add_u32 chain
            asm volatile(REP64("v_lshl_add_u32 %0, %0, 5, %1\n") : "+v"(a) : "v"(b));
        } else if constexpr (T == 10) {  // 2 interleaved dependent chains, 3 independent chains
            asm volatile(REP64("v_add3_u32 %0, %0, %3, %4\n v_add3_u32 %1, %1, %3, %4\n v_add3_u32 %2, %2, %3, %4\n") : "+v"(a), "+v"(b), "+v"(c) : "v"(d), "v"(e));
        } else if constexpr (T == 11) {  // dependent v_xor_b32 (VOP2) chain
            asm volatile(REP64("v_xor_b32 %0, %0, %1\n") : "+v"(a) : "v"(b));
        } else if constexpr (T == 12) {  // dependent v_add_u32 via DPP? no: v_add_co_u32 VOP2
            asm volatile(REP64("v_add_co_u32 %0, vcc, %0, %1\n") : "+v"(a) : "v"(b) : "vcc");
        } else if constexpr (T == 13) {  // 6 independent add3 chains
            asm volatile(REP64("v_add3_u32 %0, %0, %6, %7\n v_add3_u32 %1, %1, %6, %7\n v_add3_u32 %2, %2, %6, %7\n v_add3_u32 %3, %3, %6, %7\n v_add3_u32 %4, %4, %6, %7\n v_add3_u32 %5, %5, %6, %7\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f) : "v"(g), "v"(h));
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

static const char* names[] = {"dep add3", "dep alignbit", "dep add_u32(VOP2)", "dep bitop3", "alt alignbit->add3",
                              "4x indep add3", "8x indep alignbit", "8x indep bitop3", "2 chains add3 interleaved",
                              "dep lshl_add", "3 chains add3", "dep xor(VOP2)", "dep add_co(VOP2)", "6x indep add3"};
static const int ninstr[] = {64, 64, 64, 64, 128, 256, 512, 512, 128, 64, 192, 64, 64, 384};

template <int T>
void run(int waves_per_block, int blocks) {
    uint64_t* cyc;
    uint32_t* sink;
    hipMalloc(&cyc, sizeof(uint64_t) * blocks * waves_per_block);
    hipMalloc(&sink, 4 * blocks * waves_per_block * 64);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(kbench<T>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, cyc, sink, 1u);
        hipDeviceSynchronize();
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kbench<T>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, cyc, sink, 1u);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(blocks * waves_per_block);
    hipMemcpy(h.data(), cyc, 8 * h.size(), hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += v;
    s /= h.size();
    const double instr = 16.0 * ninstr[T];
    // wall-clock based: total instr per wave / time -> effective ns per instr
    printf("%-28s waves/blk=%d blocks=%4d : %6.2f memtime-cyc/instr   wall %.3f ms  (%.2f ns/instr/wave)\n", names[T],
           waves_per_block, blocks, s / instr, ms, ms * 1e6 / instr);
    hipFree(cyc);
    hipFree(sink);
}

template <int T>
void sweep() {
    run<T>(1, 256);    // 1 wave per CU
    run<T>(4, 256);    // ~1 wave per SIMD
    run<T>(8, 256);    // ~2 waves per SIMD
    run<T>(16, 256);   // ~4 waves per SIMD
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("device %s clock %d kHz CUs %d\n", p.name, p.clockRate, p.multiProcessorCount);
    sweep<0>(); sweep<1>(); sweep<2>(); sweep<3>(); sweep<4>(); sweep<5>(); sweep<6>();
    sweep<7>(); sweep<8>(); sweep<9>(); sweep<10>(); sweep<11>(); sweep<12>(); sweep<13>();
    return 0;
}
