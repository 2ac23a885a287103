// tools/ubench_mix_mw.hip -- does a SIMD shared by several waves run a MIX of half-rate (v_alignbit_b32, v_add3_u32,
// ~4 cycles per wave64 instruction) and full-rate (v_bitop3_b32, v_xor_b32, ~2-2.4) instructions at the sum of
// their isolated costs?  That sum is how R_valu prices SHA-1's mix; the compression alone runs ~14 %
// above it at 4-8 waves per SIMD (profiles/r01/ubench_sha1.log).
//
// Each wave runs 8 independent chains; every chain repeats one pattern of instructions (below).  Grid: 256 x B
// workgroups of 256 threads (one wave per SIMD per workgroup), B = waves per SIMD.  SIMD time per wave64
// instruction = event time / instructions per SIMD; "model" = the pattern's mean isolated cost from
// tools/ubench_simd.hip (profiles/r01/ubench_simd.log: half 4.13, bitop3 2.35, xor 2.06 cycles at 4 waves).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_mix_mw.hip -o tools/ubench_mix_mw_bin
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP4(x) x x x x
#define ALIGN(r) "v_alignbit_b32 " #r ", " #r ", " #r ", 27\n"
#define ADD3(r) "v_add3_u32 " #r ", " #r ", %8, %9\n"
#define BITOP3(r) "v_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x96\n"
#define XOR(r) "v_xor_b32 " #r ", " #r ", %8\n"
// one step of every chain with op X: 8 instructions
#define ALL(X) X(%0) X(%1) X(%2) X(%3) X(%4) X(%5) X(%6) X(%7)
#define RUN(body) asm volatile(body : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) \
                               : "v"(k1), "v"(k2))

constexpr int ITERS = 512;

// patterns (per chain, repeated): 0 add3+bitop3, 1 alignbit+xor, 2 alignbit+add3+bitop3+xor,
// 3 SHA-1's proportions (alignbit 224 : add3 160 : bitop3 144 : xor 64 per compression, here 7:5:4:2 of 18),
// 4-7 each op alone (the isolated costs, measured in the same run)
template <int T>
__global__ __launch_bounds__(256) void kmix(uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u, g = a * 17u,
             h = a * 19u, k1 = seed | 1u, k2 = seed * 7u;
    for (int it = 0; it < ITERS; it++) {
        if constexpr (T == 0) RUN(REP4(ALL(ADD3) ALL(BITOP3)));
        else if constexpr (T == 1) RUN(REP4(ALL(ALIGN) ALL(XOR)));
        else if constexpr (T == 2) RUN(REP4(ALL(ALIGN) ALL(ADD3) ALL(BITOP3) ALL(XOR)));
        else if constexpr (T == 4) RUN(REP4(ALL(ALIGN) ALL(ALIGN)));
        else if constexpr (T == 5) RUN(REP4(ALL(ADD3) ALL(ADD3)));
        else if constexpr (T == 6) RUN(REP4(ALL(BITOP3) ALL(BITOP3)));
        else if constexpr (T == 7) RUN(REP4(ALL(XOR) ALL(XOR)));
        else RUN(ALL(ALIGN) ALL(ADD3) ALL(BITOP3) ALL(ALIGN) ALL(ADD3) ALL(XOR) ALL(ALIGN) ALL(BITOP3) ALL(ADD3)
                 ALL(ALIGN) ALL(BITOP3) ALL(ALIGN) ALL(ADD3) ALL(XOR) ALL(ALIGN) ALL(ADD3) ALL(BITOP3) ALL(ALIGN));
    }
    sink[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

struct Pat { const char* name; int per_iter; double model; };
// model cycles per instruction at 4 waves: half 4.13, bitop3 2.35, xor 2.06
static const Pat kPats[] = {
    {"add3 + bitop3", 64, (4.13 + 2.35) / 2},
    {"alignbit + xor", 64, (4.13 + 2.06) / 2},
    {"alignbit + add3 + bitop3 + xor", 128, (4.13 * 2 + 2.35 + 2.06) / 4},
    {"SHA-1 proportions 7:5:4:2", 144, (4.13 * 12 + 2.35 * 4 + 2.06 * 2) / 18},
    {"alignbit only", 64, 4.13}, {"add3 only", 64, 4.13}, {"bitop3 only", 64, 2.35}, {"xor only", 64, 2.06},
};

template <int T>
static void run(int per_simd) {
    const int blocks = 256 * per_simd;
    uint32_t* sink;
    (void)hipMalloc(&sink, blocks * 256 * sizeof(uint32_t));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kmix<T>, dim3(blocks), dim3(256), 0, 0, sink, 12345u);  // warm up
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kmix<T>, dim3(blocks), dim3(256), 0, 0, sink, 777u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double ns = ms * 1e6 / (double(ITERS) * kPats[T].per_iter * per_simd);
    printf("%-32s waves/SIMD=%d : %.3f ms, %.3f ns per wave64 instr = %.2f cycles at 2.1 GHz (isolated-cost model "
           "%.2f)\n", kPats[T].name, per_simd, ms, ns, ns * 2.1, kPats[T].model);
    (void)hipFree(sink);
}

int main() {
    for (int b : {1, 4, 8}) {
        run<4>(b);
        run<5>(b);
        run<6>(b);
        run<7>(b);
        run<0>(b);
        run<1>(b);
        run<2>(b);
        run<3>(b);
    }
    return 0;
}
