// tools/ubench_banks.hip -- why does a lone wave issue a dependent VOP3 chain at ~4.9 cycles but VOP2 at ~4.1?
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_banks.hip -o /tmp/ubench_banks
// Candidates: VGPR bank conflicts among the 3 source operands (bank = vgpr index mod 4), the
// 8-byte encoding (instruction fetch), or VOP3 itself.  Each case is a dependent chain of 64
// instructions on physical registers (init moves included, identical across cases), 16 times,
// timed with s_memtime per wave; one wave per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))
#define INIT "v_mov_b32 v40, %1\n v_mov_b32 v41, %1\n v_mov_b32 v42, %1\n v_mov_b32 v43, %1\n" \
             "v_mov_b32 v44, %1\n v_mov_b32 v48, %1\n v_mov_b32 v45, %1\n v_mov_b32 v46, %1\n"
#define TAIL "v_mov_b32 %0, v40\n"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53"

template <int T>
__global__ void kbank(uint64_t* cyc, uint32_t* sink, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, r = 0;
    uint64_t t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int it = 0; it < 16; it++) {
        uint32_t o;
        if constexpr (T == 0)   // add3, sources in banks 0,1,2
            asm volatile(INIT REP64("v_add3_u32 v40, v40, v41, v42\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 1)   // add3, all sources bank 0
            asm volatile(INIT REP64("v_add3_u32 v40, v40, v44, v48\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 2)   // add3, two sources bank 0
            asm volatile(INIT REP64("v_add3_u32 v40, v40, v44, v41\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 3)   // bitop3 banks 0,1,2
            asm volatile(INIT REP64("v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 4)   // bitop3 all bank 0
            asm volatile(INIT REP64("v_bitop3_b32 v40, v40, v44, v48 bitop3:0x96\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 5)   // alignbit rotate (same reg twice)
            asm volatile(INIT REP64("v_alignbit_b32 v40, v40, v40, 27\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 6)   // alignbit, 2 distinct regs in banks 0,1
            asm volatile(INIT REP64("v_alignbit_b32 v40, v40, v41, 27\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 7)   // VOP2 add
            asm volatile(INIT REP64("v_add_u32 v40, v40, v41\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 8)   // VOP2 add with 32-bit literal (8 bytes)
            asm volatile(INIT REP64("v_add_u32 v40, 0x12345678, v40\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 9)   // same op, VOP3 encoding (8 bytes)
            asm volatile(INIT REP64("v_add_u32_e64 v40, v40, v41\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 10)  // add3 with an inline constant (2 VGPR sources)
            asm volatile(INIT REP64("v_add3_u32 v40, v40, 5, v41\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 11)  // alternating VOP3 alignbit / VOP2 add (the round's mix)
            asm volatile(INIT REP64("v_alignbit_b32 v41, v40, v40, 27\n v_add_u32 v40, v41, v42\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 12)  // 4 independent add3, distinct banks
            asm volatile(INIT REP64("v_add3_u32 v40, v40, v45, v46\n v_add3_u32 v41, v41, v44, v46\n"
                                    "v_add3_u32 v42, v42, v44, v45\n v_add3_u32 v43, v43, v45, v46\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 13)  // s_nop between dependent VOP2 adds (cost of a non-VALU slot)
            asm volatile(INIT REP64("v_add_u32 v40, v40, v41\n s_nop 0\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 14)  // VOP2 add + independent ds_read_b128 (LDS slot cost)
            asm volatile(INIT "v_mov_b32 v49, 0\n" REP64("v_add_u32 v40, v40, v41\n ds_read_b128 v[50:53], v49\n")
                         "s_waitcnt lgkmcnt(0)\n" TAIL : "=v"(o) : "v"(a) : CLOB);
        else if constexpr (T == 15)  // bfi (Ch) banks 0,1,2
            asm volatile(INIT REP64("v_bfi_b32 v40, v40, v41, v42\n") TAIL : "=v"(o) : "v"(a) : CLOB);
        r ^= o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static const char* names[] = {
    "add3 banks 0,1,2", "add3 banks 0,0,0", "add3 banks 0,0,1", "bitop3 banks 0,1,2", "bitop3 banks 0,0,0",
    "alignbit x,x", "alignbit x,y", "VOP2 add", "VOP2 add + literal (8B)", "add_u32_e64 (VOP3 enc)",
    "add3 with inline const", "alt alignbit/VOP2 add", "4x indep add3", "VOP2 add + s_nop", "VOP2 add + ds_read_b128",
    "bfi banks 0,1,2"};
static const int per_rep[] = {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 128, 256, 128, 128, 64};

template <int T>
void run(int waves_per_block) {
    const int blocks = 256;
    uint64_t* cyc;
    uint32_t* sink;
    hipMalloc(&cyc, sizeof(uint64_t) * blocks * waves_per_block);
    hipMalloc(&sink, 4 * blocks * waves_per_block * 64);
    uint64_t best = ~0ull;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(kbank<T>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, cyc, sink, 1u);
        hipDeviceSynchronize();
        uint64_t h[4 * 256];
        hipMemcpy(h, cyc, 8 * blocks * waves_per_block, hipMemcpyDeviceToHost);
        uint64_t s = 0;
        for (int i = 0; i < blocks * waves_per_block; i++) s += h[i];
        s /= blocks * waves_per_block;
        if (rep && s < best) best = s;
    }
    const double instr = 16.0 * (per_rep[T] + 9);   // + 8 init moves + 1 tail move per statement
    printf("%-26s waves/CU=%d : %5.2f cyc/instr (per wave)\n", names[T], waves_per_block, best / instr);
    hipFree(cyc);
    hipFree(sink);
}

template <int T>
void both() { run<T>(1); run<T>(4); }

int main() {
    both<0>(); both<1>(); both<2>(); both<3>(); both<4>(); both<5>(); both<6>(); both<7>();
    both<8>(); both<9>(); both<10>(); both<11>(); both<12>(); both<13>(); both<14>(); both<15>();
    return 0;
}
