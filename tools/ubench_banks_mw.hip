// tools/ubench_banks_mw.hip -- do VGPR bank conflicts among a VOP3's three sources cost SIMD throughput when
// several waves share a SIMD?  (tools/ubench_banks.hip asked it for a lone wave, whose 4-cycle issue cadence
// hides them; the saturated lane kernel runs 4 waves per SIMD at ~83 % of the op-mix model)
//
// Each wave runs 8 independent chains of one 3-source op on explicit VGPRs: chain k's destination is v(64+k);
// its two other sources are v(48+...) constants chosen either in three DIFFERENT banks (bank = index mod 4) or all
// in the SAME bank as the destination.  Grid: 256 x B workgroups of 256 threads (one wave per SIMD per
// workgroup), B = waves per SIMD.  SIMD time per wave64 instruction = event time / instructions per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_banks_mw.hip -o /tmp/ubench_banks_mw
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(x) x x x x x x x x
// chain k: destination v(64+k) (bank k mod 4); DIFF: the other sources in banks k+1 and k+2; SAME: both in bank k
#define DIFF_BITOP3(k, d, s1, s2) "v_bitop3_b32 v" #d ", v" #d ", v" #s1 ", v" #s2 " bitop3:0x96\n"
#define DIFF_ADD3(k, d, s1, s2) "v_add3_u32 v" #d ", v" #d ", v" #s1 ", v" #s2 "\n"
// eight chains: (dst, different-bank sources) and (dst, same-bank sources)
#define CHAINS_DIFF(OP) OP(0, 64, 49, 54) OP(1, 65, 50, 55) OP(2, 66, 51, 52) OP(3, 67, 48, 53) \
                        OP(4, 68, 49, 54) OP(5, 69, 50, 55) OP(6, 70, 51, 52) OP(7, 71, 48, 53)
#define CHAINS_SAME(OP) OP(0, 64, 48, 56) OP(1, 65, 49, 57) OP(2, 66, 50, 58) OP(3, 67, 51, 59) \
                        OP(4, 68, 48, 56) OP(5, 69, 49, 57) OP(6, 70, 50, 58) OP(7, 71, 51, 59)
#define INIT "v_mov_b32 v48, %0\n v_mov_b32 v49, %0\n v_mov_b32 v50, %0\n v_mov_b32 v51, %0\n" \
             "v_mov_b32 v52, %0\n v_mov_b32 v53, %0\n v_mov_b32 v54, %0\n v_mov_b32 v55, %0\n" \
             "v_mov_b32 v56, %0\n v_mov_b32 v57, %0\n v_mov_b32 v58, %0\n v_mov_b32 v59, %0\n" \
             "v_mov_b32 v64, %0\n v_mov_b32 v65, %0\n v_mov_b32 v66, %0\n v_mov_b32 v67, %0\n" \
             "v_mov_b32 v68, %0\n v_mov_b32 v69, %0\n v_mov_b32 v70, %0\n v_mov_b32 v71, %0\n"
#define CLOB "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", \
             "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71"

constexpr int ITERS = 1024;  // x 64 instructions per wave

template <int T>
__global__ __launch_bounds__(256) void kbench(uint64_t* cyc, uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, o = 0;
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile(INIT ::"v"(a) : CLOB);
    for (int it = 0; it < ITERS; it++) {
        if constexpr (T == 0) asm volatile(REP8(CHAINS_DIFF(DIFF_BITOP3)) ::: CLOB);
        else if constexpr (T == 1) asm volatile(REP8(CHAINS_SAME(DIFF_BITOP3)) ::: CLOB);
        else if constexpr (T == 2) asm volatile(REP8(CHAINS_DIFF(DIFF_ADD3)) ::: CLOB);
        else asm volatile(REP8(CHAINS_SAME(DIFF_ADD3)) ::: CLOB);
    }
    asm volatile("v_xor_b32 %0, v64, v71" : "=v"(o)::CLOB);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * 256 + threadIdx.x] = o;
}

static const char* kNames[] = {"v_bitop3_b32, sources in 3 banks", "v_bitop3_b32, sources in 1 bank",
                               "v_add3_u32, sources in 3 banks", "v_add3_u32, sources in 1 bank"};

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
    uint64_t c0 = 0;
    (void)hipMemcpy(&c0, cyc, sizeof c0, hipMemcpyDeviceToHost);
    const double instr_per_wave = double(ITERS) * 64.0;
    // SIMD time per wave64 instruction from the launch's event time (every SIMD runs per_simd waves)
    const double ns_per_instr = ms * 1e6 / (instr_per_wave * per_simd);
    printf("%-36s waves/SIMD=%d : %.3f ms, SIMD %.3f ns per wave64 instr (= %.2f cycles at 2.1 GHz)\n", kNames[T],
           per_simd, ms, ns_per_instr, ns_per_instr * 2.1);
    (void)hipFree(cyc);
    (void)hipFree(sink);
}

int main() {
    for (int b : {1, 4, 8}) {
        run<0>(b);
        run<1>(b);
        run<2>(b);
        run<3>(b);
    }
    return 0;
}
