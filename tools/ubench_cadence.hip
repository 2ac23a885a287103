// tools/ubench_cadence.hip -- what sets a lone wave's issue cadence for 8-byte VALU instructions?
//
// Round 1 left two readings: ubench_fetch (independent v_add3 chains in a 64-B-aligned loop) issued at
// 4.07 cycles per instruction, while ubench_simd / ubench_banks (the same kind of stream, compiler-placed)
// gave 4.58-4.98.  Round 2's DESIGN explained the lane kernel by the second number (instruction bytes).
// This probe runs ONE wave per CU over the same 4-chain v_add3 stream in different code layouts and reports
// s_memtime cycles per VALU instruction:
//   loop_a64   : 512 add3 per trip, loop top .p2align 6            (ubench_fetch's layout)
//   loop_a64p4 : same, loop top at 64n + 4
//   loop_a64p32: same, loop top at 64n + 32
//   lit8       : 512 VOP2 v_add_u32 with a 32-bit literal (8 B) per trip, aligned
//   vop2       : 512 VOP2 v_add_u32 (4 B) per trip, aligned
//   mix36      : the SHA-1 round mix (rotl5, e+KW VOP2, f, add3, rotl30 = 36 B per round), 80 rounds/trip
//   line       : 2,048 add3 straight-line (16 KiB, no loop), executed once -- cold instruction cache
//   line2      : the same 16 KiB straight-line block executed twice in a row (a 2-trip loop) -- warm second trip
//   dep1       : 512 add3 per trip, 1 chain (each depends on the previous)
//   dep2       : 512 add3 per trip, 2 interleaved chains
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_cadence.hip -o build/ubench_cadence
#include <hip/hip_runtime.h>

#include <cstdio>

#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)
#define R16(x) R8(x) R8(x)
#define R32(x) R16(x) R16(x)
#define R64(x) R32(x) R32(x)
#define R128(x) R64(x) R64(x)
#define R512(x) R4(R128(x))

#define A4 "v_add3_u32 v40, v40, v44, v45\n v_add3_u32 v41, v41, v44, v45\n" \
           "v_add3_u32 v42, v42, v44, v45\n v_add3_u32 v43, v43, v44, v45\n"
#define D1 "v_add3_u32 v40, v40, v44, v45\n"
#define D2 "v_add3_u32 v40, v40, v44, v45\n v_add3_u32 v41, v41, v44, v45\n"
#define L8 "v_add_u32 v40, 0x12345678, v40\n v_add_u32 v41, 0x12345678, v41\n" \
           "v_add_u32 v42, 0x12345678, v42\n v_add_u32 v43, 0x12345678, v43\n"
#define V4 "v_add_u32 v40, v44, v40\n v_add_u32 v41, v44, v41\n v_add_u32 v42, v44, v42\n v_add_u32 v43, v44, v43\n"
#define ROUND "v_alignbit_b32 v46, v40, v40, 27\n v_add_u32 v47, v43, v44\n" \
              "v_bitop3_b32 v48, v41, v42, v43 bitop3:0x96\n v_add3_u32 v40, v46, v48, v47\n" \
              "v_alignbit_b32 v42, v41, v41, 2\n"

#define PRE(trips) "s_mov_b32 s40, " #trips "\n" \
    "v_mov_b32 v40, %1\n v_mov_b32 v41, %1\n v_mov_b32 v42, %1\n v_mov_b32 v43, %1\n" \
    "v_mov_b32 v44, %1\n v_mov_b32 v45, %1\n v_mov_b32 v46, %1\n v_mov_b32 v47, %1\n v_mov_b32 v48, %1\n"
#define POST "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 L_top_%=\n v_mov_b32 %0, v40\n"
#define CLOB "s40", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "scc"

// loop, top aligned to 64 B plus `pad` bytes of s_nop (outside the loop)
#define LOOP(body, trips, pad) \
    asm volatile(PRE(trips) "s_branch L_top_%=\n .p2align 6\n" pad "L_top_%=:\n" body POST : "=v"(o) : "v"(a) : CLOB)

template <int T>
__global__ void kcad(uint64_t* cyc, uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, o;
    uint64_t t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    if constexpr (T == 0) LOOP(R128(A4), 32, "");
    else if constexpr (T == 1) LOOP(R128(A4), 32, "s_nop 0\n");
    else if constexpr (T == 2) LOOP(R128(A4), 32, R8("s_nop 0\n"));
    else if constexpr (T == 3) LOOP(R128(L8), 32, "");
    else if constexpr (T == 4) LOOP(R128(V4), 32, "");
    else if constexpr (T == 5) LOOP(R64(ROUND) R16(ROUND), 40, "");
    else if constexpr (T == 6) LOOP(R512(A4), 1, "");
    else if constexpr (T == 7) LOOP(R512(A4), 2, "");
    else if constexpr (T == 8) LOOP(R512(D1), 32, "");
    else LOOP(R128(R2(D2)), 32, "");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = o;
}

static const char* names[] = {"loop_a64", "loop_a64p4", "loop_a64p32", "lit8", "vop2", "mix36", "line", "line2",
                              "dep1", "dep2"};
static const int per_trip[] = {512, 512, 512, 512, 512, 400, 2048, 2048, 512, 512};
static const int trips[] = {32, 32, 32, 32, 32, 40, 1, 2, 32, 32};

template <int T>
void run() {
    const int blocks = 256;
    uint64_t* cyc;
    uint32_t* sink;
    (void)hipMalloc(&cyc, sizeof(uint64_t) * blocks);
    (void)hipMalloc(&sink, 4 * blocks * 64);
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {
        hipLaunchKernelGGL(kcad<T>, dim3(blocks), dim3(64), 0, 0, cyc, sink, 1u);
        (void)hipDeviceSynchronize();
        uint64_t h[256];
        (void)hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; i++) s += (double)h[i];
        s /= blocks;
        if (rep && s < best) best = s;
    }
    const double valu = (double)per_trip[T] * trips[T];
    printf("%-12s : %5.2f cyc per VALU instr (incl. loop overhead), %8.1f cyc per trip\n", names[T], best / valu,
           best / trips[T]);
    (void)hipFree(cyc);
    (void)hipFree(sink);
}

int main() {
    run<0>(); run<1>(); run<2>(); run<3>(); run<4>(); run<5>(); run<6>(); run<7>(); run<8>(); run<9>();
    return 0;
}
