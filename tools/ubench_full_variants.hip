// tools/ubench_full_variants.hip -- which part of the full compression runs slower than a lone wave's
// 4.07-cycle cadence?  Timing-only variants of the generated tv_sha1_full (results are not SHA-1):
//   a  as generated (592 VALU)
//   b  schedule xor3 (v_bitop3 0x96, 3 VGPR sources) -> VOP2 v_xor (2 sources)
//   c  schedule rotl1 (v_alignbit w,w,w,31) -> VOP2 v_lshlrev
//   d  b + c
//   e  rounds only (schedule removed, 400 VALU)
//   f  a with K in VGPRs     g  e with K in VGPRs
//   h  e with e+K+W as VOP2 v_add e, W (K dropped)     i  a with the same VOP2 e + W
//   j-m  tools/gen_full_sched.py pipelined schedules (real SHA-1): lag 1 plain, lag 1/2/3 f_first
//   n  e with e+K+W as v_add_u32_e64 e, W   o  e with v_add3 e, W, 0   p  a with v_add_u32_e64 e, W
//   q  real SHA-1: e+K+W as two VOP2 adds (tools/gen_full_sched.py gen_full_kw_vop2, 672 VALU)
//   r  e with e+K+W after the rotl5   s  e with s_nop 0 after e+K+W   t  e with a VOP2 v_mov after e+K+W
//   base / u  the lane kernel's bswap + compress, with the next block's 16 v_perm outside / inside rounds 0-15
// Build: python3 tools/ubench_full_variants.py <dir> (writes <dir>/variants.h), then
//   hipcc --offload-arch=gfx950 -O3 -I <dir of variants.h> tools/ubench_full_variants.hip -o tools/ubench_full_variants_bin
// One wave per CU, two compressions per loop trip; cycles per compression from block 0's s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "variants.h"

#define KERNEL(V)                                                                               \
__global__ __launch_bounds__(64) void k_##V(uint32_t* out, int iters, uint64_t* clk) {          \
    uint32_t h[5] = {threadIdx.x, 2, 3, 4, 5};                                                  \
    uint32_t w[16];                                                                             \
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * (i + 1);                                  \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
    for (int it = 0; it < iters; it += 2) {                                                     \
        uint32_t r[5];                                                                          \
        tv_sha1_full_##V(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);          \
        for (int i = 0; i < 5; i++) h[i] += r[i];                                               \
        tv_sha1_full_##V(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);          \
        for (int i = 0; i < 5; i++) h[i] += r[i];                                               \
    }                                                                                           \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
    out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ w[3];               \
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                            \
}
KERNEL(a) KERNEL(b) KERNEL(c) KERNEL(d) KERNEL(e) KERNEL(f) KERNEL(g) KERNEL(h) KERNEL(i) KERNEL(j) KERNEL(k) KERNEL(l) KERNEL(m) KERNEL(n) KERNEL(o) KERNEL(p) KERNEL(q) KERNEL(r) KERNEL(s) KERNEL(t)

// the lane kernel's shape: raw (little-endian) words of the next block -> bswap -> compress.
// base: 16 v_perm outside the asm before each compression; u: the next block's v_perm inside the
// previous compression's rounds 0-15 (ping-pong w buffers, so no register copies)
__device__ __forceinline__ uint32_t bs(uint32_t x) { return __builtin_amdgcn_perm(0, x, 0x00010203u); }
__global__ __launch_bounds__(64) void k_base(uint32_t* out, int iters, uint64_t* clk) {
    uint32_t h[5] = {threadIdx.x, 2, 3, 4, 5};
    uint32_t x[16], w[16];
    for (int i = 0; i < 16; i++) x[i] = threadIdx.x * (i + 7) + i;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it += 2) {
        uint32_t r[5];
        for (int i = 0; i < 16; i++) w[i] = bs(x[i] + it);
        tv_sha1_full_a(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
        for (int i = 0; i < 16; i++) w[i] = bs(x[i] ^ it);
        tv_sha1_full_a(h, r, w, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ w[3];
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ __launch_bounds__(64) void k_u(uint32_t* out, int iters, uint64_t* clk) {
    uint32_t h[5] = {threadIdx.x, 2, 3, 4, 5};
    uint32_t x[16], wa[16], wb[16], xa[16], xb[16];
    for (int i = 0; i < 16; i++) { x[i] = threadIdx.x * (i + 7) + i; wa[i] = bs(x[i]); }
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it += 2) {
        uint32_t r[5];
        for (int i = 0; i < 16; i++) xa[i] = x[i] + it;      // stands in for the next block's loads
        tv_sha1_full_u(h, r, wa, xa, wb, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
        for (int i = 0; i < 16; i++) xb[i] = x[i] ^ it;
        tv_sha1_full_u(h, r, wb, xb, wa, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u);
        for (int i = 0; i < 5; i++) h[i] += r[i];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ wa[3];
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

typedef void (*kfn)(uint32_t*, int, uint64_t*);

int main() {
    uint32_t* out; uint64_t* clk;
    if (hipMalloc(&out, 4 << 20) != hipSuccess || hipMalloc(&clk, 8 * 256) != hipSuccess) return 1;
    const int iters = 2000;
    struct { const char* name; kfn f; int valu; } v[] = {
        {"a as generated", k_a, 597}, {"b xor3 -> VOP2 xor", k_b, 597}, {"c rotl1 -> VOP2 lshl", k_c, 597},
        {"d b + c", k_d, 597}, {"e rounds only", k_e, 405},
        {"f a, K in VGPR", k_f, 597}, {"g e, K in VGPR", k_g, 405}, {"h e, VOP2 e+W", k_h, 405},
        {"i a, VOP2 e+W", k_i, 597}, {"j lag1 plain", k_j, 597}, {"k lag1 f_first", k_k, 597},
        {"l lag2 f_first", k_l, 597}, {"m lag3 f_first", k_m, 597}, {"n e, VOP3 add_e64 e+W", k_n, 405},
        {"o e, add3 e,W,0", k_o, 405}, {"p a, VOP3 add_e64 e+W", k_p, 597},
        {"q real: kw=K+W, e+=kw VOP2", k_q, 677}, {"r e, e+K+W after rotl5", k_r, 405},
        {"s e, s_nop after e+K+W", k_s, 405}, {"t e, VOP2 mov after e+K+W", k_t, 485},
        {"base: bswap outside", k_base, 629}, {"u: next bswap inside", k_u, 629}};
    for (int rep = 0; rep < 2; rep++)
        for (auto& x : v) {
            hipLaunchKernelGGL(x.f, dim3(256), dim3(64), 0, 0, out, 50, clk);
            hipLaunchKernelGGL(x.f, dim3(256), dim3(64), 0, 0, out, iters, clk);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            uint64_t c = 0;
            if (hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
            printf("%-22s cycles per compression %6.0f   %.3f per VALU (%d)\n", x.name, (double)c / iters,
                   (double)c / iters / x.valu, x.valu);
        }
    return 0;
}
