// tools/ubench_fetch.hip -- does a lone wave issue 8-byte VALU instructions faster from a SMALL loop?
//
// ubench_banks.hip found a lone wave issuing DEPENDENT chains of 8-byte instructions at 4.93 cyc
// (≈ 1.62 instruction bytes per cycle) against 4.11 cyc for 4-byte ones, which read like an
// instruction-fetch bound.  This probe answers it: independent 8-byte instructions in loops of K per
// trip (trips x K = 16,384), and the SHA-1 round mix, one wave per CU, timed by s_memtime, reported
// per VALU instruction.  Result (profiles/r01/ubench_fetch.log): 4.07 cyc for long bodies, so there
// is no fetch bound; the 4.93 is the back-to-back VOP3 dependency.  Also: an SGPR source costs nothing.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_fetch.hip -o tools/ubench_fetch
#include <hip/hip_runtime.h>

#include <cstdio>

#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)
#define R16(x) R8(x) R8(x)
#define R32(x) R16(x) R16(x)
#define R64(x) R32(x) R32(x)
#define R128(x) R64(x) R64(x)

// 8-byte VOP3, 4 independent chains (no dependency stall at any issue rate)
#define V8 "v_add3_u32 v40, v40, v44, v45\n v_add3_u32 v41, v41, v44, v45\n" \
           "v_add3_u32 v42, v42, v44, v45\n v_add3_u32 v43, v43, v44, v45\n"
// one SHA-1 round's mix: rotl5 (8B), e+KW (4B VOP2), f (8B), sum (8B), rotl30 (8B) = 36 B
#define ROUND "v_alignbit_b32 v46, v40, v40, 27\n v_add_u32 v47, v43, v44\n" \
              "v_bitop3_b32 v48, v41, v42, v43 bitop3:0x96\n v_add3_u32 v40, v46, v48, v47\n" \
              "v_alignbit_b32 v42, v41, v41, 2\n"

// 8-byte VOP3 with an SGPR source (the lane kernel's e + K + W with K in an SGPR) vs the same with
// the constant in a VGPR
#define V8S "v_add3_u32 v40, v40, s44, v45\n v_add3_u32 v41, v41, s44, v45\n" \
            "v_add3_u32 v42, v42, s44, v45\n v_add3_u32 v43, v43, s44, v45\n"
#define V8V "v_add3_u32 v40, v40, v46, v45\n v_add3_u32 v41, v41, v46, v45\n" \
            "v_add3_u32 v42, v42, v46, v45\n v_add3_u32 v43, v43, v46, v45\n"
// the round mix with e + K + W as one v_add3 (K in an SGPR / in a VGPR) instead of a VOP2 add
#define ROUNDS "v_alignbit_b32 v46, v40, v40, 27\n v_add3_u32 v47, v43, s44, v44\n" \
               "v_bitop3_b32 v48, v41, v42, v43 bitop3:0x96\n v_add3_u32 v40, v46, v48, v47\n" \
               "v_alignbit_b32 v42, v41, v41, 2\n"
#define ROUNDV "v_alignbit_b32 v46, v40, v40, 27\n v_add3_u32 v47, v43, v45, v44\n" \
               "v_bitop3_b32 v48, v41, v42, v43 bitop3:0x96\n v_add3_u32 v40, v46, v48, v47\n" \
               "v_alignbit_b32 v42, v41, v41, 2\n"

#define LOOP(body, trips)                                                                    \
    asm volatile("s_mov_b32 s40, " #trips "\n"                                                     \
                 "v_mov_b32 v40, %1\n v_mov_b32 v41, %1\n v_mov_b32 v42, %1\n v_mov_b32 v43, %1\n" \
                 "v_mov_b32 v44, %1\n v_mov_b32 v45, %1\n v_mov_b32 v46, %1\n s_mov_b32 s44, 0x5a827999\n" \
                 "s_branch L_top_%=\n"                                                        \
                 ".p2align 6\n"                                                                    \
                 "L_top_%=:\n" body                                                           \
                 "s_sub_u32 s40, s40, 1\n"                                                         \
                 "s_cmp_lg_u32 s40, 0\n"                                                           \
                 "s_cbranch_scc1 L_top_%=\n"                                                  \
                 "v_mov_b32 %0, v40\n"                                                             \
                 : "=v"(o) : "v"(a) : "s40", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "s44", "scc")

template <int T>
__global__ void kfetch(uint64_t* cyc, uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, o;
    uint64_t t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    if constexpr (T == 0) LOOP(V8, 4096);                  // 4 instr / trip (32 B)
    else if constexpr (T == 1) LOOP(R2(V8), 2048);         // 8 (64 B)
    else if constexpr (T == 2) LOOP(R4(V8), 1024);         // 16 (128 B)
    else if constexpr (T == 3) LOOP(R8(V8), 512);          // 32 (256 B)
    else if constexpr (T == 4) LOOP(R16(V8), 256);         // 64 (512 B)
    else if constexpr (T == 5) LOOP(R64(V8), 64);          // 256 (2 KiB)
    else if constexpr (T == 6) LOOP(R128(V8), 32);         // 512 (4 KiB)
    else if constexpr (T == 7) LOOP(ROUND, 3200);          // 5 instr / trip: one round (36 B)
    else if constexpr (T == 8) LOOP(R4(ROUND), 800);       // 4 rounds (144 B)
    else if constexpr (T == 9) LOOP(R16(ROUND), 200);      // 16 rounds (576 B)
    else if constexpr (T == 10) LOOP(R32(R2(ROUND)) R16(ROUND), 40);   // 80 rounds (2,880 B)
    else if constexpr (T == 11) LOOP(R128(V8S), 32);       // 512 add3 with an SGPR source
    else if constexpr (T == 12) LOOP(R128(V8V), 32);       // 512 add3, all VGPR sources
    else if constexpr (T == 13) LOOP(R32(R2(ROUNDS)) R16(ROUNDS), 40);  // 80 rounds, e+K+W = add3 (K in SGPR)
    else LOOP(R32(R2(ROUNDV)) R16(ROUNDV), 40);            // 80 rounds, e+K+W = add3 (K in VGPR)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = o;
}

static const char* names[] = {"8B x4 / trip", "8B x8 / trip", "8B x16 / trip", "8B x32 / trip", "8B x64 / trip",
                              "8B x256 / trip", "8B x512 / trip", "round x1 / trip", "round x4 / trip",
                              "round x16 / trip", "round x80 / trip", "add3 sgpr x512", "add3 vgpr x512",
                              "round80 K sgpr", "round80 K vgpr"};
static const int per_trip[] = {4, 8, 16, 32, 64, 256, 512, 5, 20, 80, 400, 512, 512, 400, 400};
static const int trips[] = {4096, 2048, 1024, 512, 256, 64, 32, 3200, 800, 200, 40, 32, 32, 40, 40};

template <int T>
void run() {
    const int blocks = 256;
    uint64_t* cyc;
    uint32_t* sink;
    (void)hipMalloc(&cyc, sizeof(uint64_t) * blocks);
    (void)hipMalloc(&sink, 4 * blocks * 64);
    double best = 1e30;
    for (int rep = 0; rep < 4; rep++) {
        hipLaunchKernelGGL(kfetch<T>, dim3(blocks), dim3(64), 0, 0, cyc, sink, 1u);
        (void)hipDeviceSynchronize();
        uint64_t h[256];
        (void)hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; i++) s += (double)h[i];
        s /= blocks;
        if (rep && s < best) best = s;
    }
    const double valu = (double)per_trip[T] * trips[T];
    printf("%-18s : %5.2f cyc per VALU instr (incl. loop overhead), %7.1f cyc per trip\n", names[T], best / valu,
           best / trips[T]);
    (void)hipFree(cyc);
    (void)hipFree(sink);
}

int main() {
    run<0>(); run<1>(); run<2>(); run<3>(); run<4>(); run<5>(); run<6>();
    run<7>(); run<8>(); run<9>(); run<10>(); run<11>(); run<12>(); run<13>(); run<14>();
    return 0;
}
