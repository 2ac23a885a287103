// tv_kernels.hip -- gfx950 SHA-1 piece-verification kernels.
//
// Reference semantics (rclarey/torrent): piece i = bytes [i*L, i*L + len_i) of the linear
// torrent space (torrent.ts:165,186); len_i per piece.ts:16-19; digest = SHA-1 as in
// crypto.subtle.digest("SHA-1", content) (tools/make_torrent.ts:28-31); have-bit i set iff
// the digest equals info.pieces[i] (metainfo.ts:111) and the bytes were readable
// (Storage.get non-null, storage.ts:50-65), MSB-first (torrent.ts:147-149).
//
// SHA-1 is serial inside a piece, so parallelism comes from pieces only.  Three kernels (plus list modes):
//   lane  : one lane per piece; each lane loads its own 64-byte blocks (register prefetch, TV_LANE_DEPTH = 3
//           blocks ahead) and runs the full compression (schedule + rounds) as one generated asm block
//           (613 VALU per block).  For > 32,768 pieces per GPU, where every SIMD has a wave.
//   split : schedule offload.  A workgroup is PAIRS x (rounds, helper) waves, 64 pieces per pair: a helper
//           loads the blocks and writes K+W[0..79] into a 3-buffer LDS ring two blocks ahead (generated asm:
//           v_perm bswap, v_bitop3 xor3, K adds, ds_write_b128); the rounds wave runs only the 80 rounds
//           from LDS (405 VALU + 20 ds_read_b128 + 5 waits per block).  A lone wave issues one VALU per
//           ~4.07 cycles (tools/ubench_fetch.hip), so with fewer pieces than SIMDs the per-lane
//           instruction count IS the bound; this cuts the serial stream from 613 to 405 VALU per block.
//           For 16,384 < pieces <= 32,768 per GPU.
//   twin  : split with TWO lanes per piece: a lane pair runs the same rounds, each lane reads only the K+W
//           quads of its parity (10 ds_read_b128 per block) and takes the other parity's word from its
//           partner by DPP; a two-lane helper expands the schedule by parity.  For <= 16,384 pieces per GPU
//           (every wave still has a SIMD to itself).
//
// HBM layout: resident piece j (shard-local) starts at payload + j*stride, stride = L + pad
// (pad breaks the power-of-two stride that would put all 64 lanes of a wave on one channel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha1_asm.h"
#include "tv_internal.h"

#define TV_K0 0x5A827999u
#define TV_K1 0x6ED9EBA1u
#define TV_K2 0x8F1BBCDCu
#define TV_K3 0xCA62C1D6u

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void sha1_iv(uint32_t h[5]) {
    h[0] = 0x67452301u; h[1] = 0xEFCDAB89u; h[2] = 0x98BADCFEu; h[3] = 0x10325476u; h[4] = 0xC3D2E1F0u;
}

// Per-wave uniform geometry.  Every piece of a launch has length L except the global last
// piece (launch-local index last_idx), which is always the final piece of the launch.  All
// values are made provably wave-uniform (readfirstlane) so loop control stays scalar and the
// prefetch loads are never predicated (a predicated load forces a vmcnt(0) + copy at the join).
struct WaveGeom {
    uint32_t fast_begin;  // first block of this launch
    uint32_t fast_end;    // blocks [fast_begin, fast_end) are raw data for EVERY lane of the wave
    uint32_t end;         // blocks [.., end) are processed (max over lanes, clipped to blk_end)
    uint32_t nb_min;      // every lane has at least nb_min blocks (no masking below it)
};

__device__ __forceinline__ uint64_t nblocks(uint64_t len) { return (len + 8) / 64 + 1; }

__device__ __forceinline__ uint32_t uni(uint64_t x) {
    return __builtin_amdgcn_readfirstlane((uint32_t)x);
}

// j0 must be wave-uniform: the first piece of the group of `span` pieces (a wave, or a split
// workgroup) that must agree on block counts.  Lanes past the launch's end are clamped to its last
// piece, so a group "has" the last piece iff last_idx falls inside [j0, j0 + span).
__device__ __forceinline__ WaveGeom wave_geom_flags(const TvPieces& p, bool has_last, bool only_last);

__device__ __forceinline__ WaveGeom wave_geom(const TvPieces& p, uint32_t j0, uint32_t span = 64) {
    // (a SHORT last piece is never in a main group: it has a dedicated group, see TvPieces::n_main)
    const bool has_last = p.last_idx < p.n_main && p.last_idx >= j0 && p.last_idx - j0 < span;
    const bool only_last = has_last && p.last_idx == j0;
    return wave_geom_flags(p, has_last, only_last);
}

// has_last: some lane's piece is the short last piece; only_last: every lane's is.
__device__ __forceinline__ WaveGeom wave_geom_flags(const TvPieces& p, bool has_last, bool only_last) {
    const uint64_t nfull_min = (has_last ? p.last_len : p.L) / 64;
    const uint64_t nb_max = nblocks(only_last ? p.last_len : p.L);
    const uint64_t nb_min = nblocks(has_last ? p.last_len : p.L);
    WaveGeom g;
    g.fast_begin = uni(p.blk_begin);
    g.fast_end = uni(nfull_min < p.blk_end ? nfull_min : p.blk_end);
    g.end = uni(nb_max < p.blk_end ? nb_max : p.blk_end);
    g.nb_min = uni(nb_min);
    return g;
}

// Build the 16 big-endian message words of block b of a piece of length len whose byte 0 is
// at `piece` (slow path: data tail, 0x80 terminator, zero fill, bit length).  Reads at most
// 64 bytes from piece + 64*b; the buffers carry >= 64 bytes of slack past every piece.
__device__ __forceinline__ void build_tail_block(const uint8_t* piece, uint64_t len, uint64_t b,
                                                 uint32_t w[16]) {
    const int64_t rem = (int64_t)len - (int64_t)(b * 64);
    uint4 raw[4];
    if (rem > 0) {
        const uint4* src = reinterpret_cast<const uint4*>(piece + b * 64);
#pragma unroll
        for (int i = 0; i < 4; i++) raw[i] = src[i];
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) raw[i] = make_uint4(0, 0, 0, 0);
    }
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(raw);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int64_t v = rem - 4 * k;  // valid data bytes in word k (may be <0 or >=4)
        uint32_t x = bswap32(rw[k]);
        if (v < 4) {
            if (v < 0) {
                x = 0;
            } else {
                const uint32_t keep = v == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * (int)v));
                x = (x & keep) | (0x80u << (24 - 8 * (int)v));
            }
        }
        w[k] = x;
    }
    if (b == nblocks(len) - 1) {
        const uint64_t bits = len * 8;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
    }
}

__device__ __forceinline__ void load_block(const uint8_t* piece, uint32_t b, uint4 (&r)[4]) {
    const uint4* src = reinterpret_cast<const uint4*>(piece + (uint64_t)b * 64);
#pragma unroll
    for (int i = 0; i < 4; i++) r[i] = src[i];
}

__device__ __forceinline__ void bswap_block(const uint4 (&r)[4], uint32_t w[16]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        w[4 * i + 0] = bswap32(r[i].x);
        w[4 * i + 1] = bswap32(r[i].y);
        w[4 * i + 2] = bswap32(r[i].z);
        w[4 * i + 3] = bswap32(r[i].w);
    }
}

__device__ __forceinline__ void compress_full(uint32_t h[5], uint32_t w[16]) {
    uint32_t r[5];
    tv_sha1_full(h, r, w, TV_K0, TV_K1, TV_K2, TV_K3);
#pragma unroll
    for (int i = 0; i < 5; i++) h[i] += r[i];
}

// Lane-local piece length.
__device__ __forceinline__ uint64_t lane_len(const TvPieces& p, uint32_t jj) {
    return jj == p.last_idx ? p.last_len : p.L;
}

// Final step shared by both kernels: compare (verify) or store (hash) the digest, or keep the
// chaining value for the next launch of a streamed run.  `writer`: this lane owns piece jj's outputs
// (a main-group lane below n_main, or lane 0 of the short last piece's dedicated group).  Bitfield
// words are OR-ed into the zeroed output (the last group may share a word with a main group).
template <bool HASH>
__device__ __forceinline__ void finish(const TvPieces& p, bool writer, uint32_t jj, uint32_t j0,
                                       const uint32_t h[5], bool last_grp) {
    if (!p.finalize) {
        if (writer) {
#pragma unroll
            for (int k = 0; k < 5; k++) p.state[(uint64_t)k * p.dcount + jj] = h[k];   // the next column's launch reads it
        }
        return;
    }
    if (HASH) {
        if (writer) {
#pragma unroll
            for (int k = 0; k < 5; k++) p.out_digests[(uint64_t)k * p.dcount + jj] = h[k];
        }
        return;
    }
    bool ok = writer;
#pragma unroll
    for (int k = 0; k < 5; k++) ok &= (h[k] == p.digests[(uint64_t)k * p.dcount + jj]);
    const uint64_t mask = __ballot(ok);
    if ((threadIdx.x & 63) == 0) {
        // ballot bit l = piece j0+l  ->  MSB-first bytes: byte m holds pieces j0+8m .. j0+8m+7
        const uint32_t w = (last_grp ? jj : j0) >> 6;
        uint64_t bits = last_grp ? ((mask & 1) ? 1ull << (((jj >> 3) & 7) * 8 + 7 - (jj & 7)) : 0)
                                 : __builtin_bswap64(__builtin_bitreverse64(mask));
        if (p.avail64) bits &= p.avail64[w];
        if (bits) atomicOr(reinterpret_cast<unsigned long long*>(p.out64 + w), (unsigned long long)bits);
    }
}

// Clock probe (TV_OPT_CLOCK_PROBE): workgroup 0 reads the shader clock counter (s_memtime) and the 100 MHz
// real-time counter (s_memrealtime) when it starts; lane 0 of its first (rounds) wave writes both pairs with a
// vector store when it ends.  The ratio of the two intervals is the shader clock the kernel actually ran at.
struct ClockStamp {
    uint64_t t0 = 0, r0 = 0;
    __device__ __forceinline__ void start(const TvPieces& p) {
        if (p.clock && blockIdx.x == 0) {   // (kernel argument and block index: a scalar branch)
            t0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
        }
    }
    __device__ __forceinline__ void end(const TvPieces& p) const {
        if (p.clock && blockIdx.x == 0 && threadIdx.x == 0) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            reinterpret_cast<ulonglong2*>(p.clock)[0] = make_ulonglong2(t0, r0);
            reinterpret_cast<ulonglong2*>(p.clock)[1] = make_ulonglong2(t1, r1);
        }
    }
};

__device__ __forceinline__ void start_state(const TvPieces& p, uint32_t jj, uint32_t h[5]) {
    if (p.blk_begin == 0) {
        sha1_iv(h);
    } else {
#pragma unroll
        for (int k = 0; k < 5; k++) h[k] = p.state[(uint64_t)k * p.dcount + jj];  // the previous column's chaining value
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// lane kernel: one lane per piece, full compression per lane.
// ------------------------------------------------------------------------------------------
#ifndef TV_LANE_DEPTH
#define TV_LANE_DEPTH 3   // raw blocks in flight per lane: 3 is 0.8-1.2 % faster than 2, 4 and 6 no better
                          // (profiles/r02/lane_depth.jsonl; A/B: tools/build_variants.py D_TV_LANE_DEPTH=n)
#endif

// Wave-group gw of a launch: pieces [64 gw, 64 gw + 64) (clamped to n_main), or, for gw == the first group
// past n_main, the short last piece alone.  Blocks [blk_begin, blk_end) of p.
// PAIRS: the raw-block loop's register ring holds 4 blocks refilled two at a time, so a lane's two 64-B blocks of
// one 128-B line are requested back to back.  With >= 1 wave per SIMD (>= 65,536 pieces on 256 CUs) the single
// loads of the 3-deep ring let ~2 % of the lines be evicted between their two halves (HBM reads 1.023 x payload
// at 262,144 x 64 KiB, L2 hit 35 %); pairs read 1.0004 x and run 0.3-2.6 % faster there, but 0.4-0.8 % slower
// below one wave per SIMD (profiles/r04/variants/ab_lane_pairs_sweep.jsonl), so the host picks (lane_pairs).
template <bool HASH, bool PAIRS>
__device__ __forceinline__ void lane_group(const TvPieces& p, uint32_t gw) {
    const uint32_t lane = threadIdx.x & 63u;
    // main waves cover [0, n_main); a short last piece (n_main < n) gets the wave after them alone
    const uint32_t nw_main = (p.n_main + 63u) / 64u;
    const bool last_grp = gw >= nw_main;
    if (last_grp && (gw > nw_main || p.n_main == p.n)) return;  // wave-uniform: no piece here
    const uint32_t j0 = last_grp ? p.last_idx : gw * 64u;
    const uint32_t j = last_grp ? p.last_idx : j0 + lane;
    const uint32_t jj = last_grp ? p.last_idx : (j < p.n_main ? j : p.n_main - 1);
    const bool writer = last_grp ? lane == 0 : j < p.n_main;
    const WaveGeom g = last_grp ? wave_geom_flags(p, true, true) : wave_geom(p, j0);
    const uint64_t len = lane_len(p, jj);
    const uint32_t nb = (uint32_t)nblocks(len);
    const uint8_t* piece = p.data + (uint64_t)jj * p.stride - p.data_off;

    uint32_t h[5];
    start_state(p, jj, h);

    uint32_t b = g.fast_begin;
    uint32_t w[16];
    if (PAIRS && b < g.fast_end) {
        // a ring of 4 register blocks refilled in pairs: a lane's two 64-B blocks of one 128-B line are loaded
        // back to back, so both halves reach L2 together
        const uint32_t last = g.fast_end - 1;
        uint4 R[4][4];
#pragma unroll
        for (int d = 0; d < 4; d++) load_block(piece, b + d < last ? b + d : last, R[d]);
        for (;;) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                bswap_block(R[2 * q], w);
                compress_full(h, w);
                if (++b >= g.fast_end) goto raw_done;
                bswap_block(R[2 * q + 1], w);
                load_block(piece, b + 3 < last ? b + 3 : last, R[2 * q]);
                load_block(piece, b + 4 < last ? b + 4 : last, R[2 * q + 1]);
                compress_full(h, w);
                if (++b >= g.fast_end) goto raw_done;
            }
        }
    }
    if (!PAIRS && b < g.fast_end) {
        // TV_LANE_DEPTH register blocks in flight.  Loads are unconditional (the block index is clamped
        // to the last raw block), so they are never predicated and stay in flight across a block.
        constexpr int D = TV_LANE_DEPTH;
        const uint32_t last = g.fast_end - 1;
        uint4 R[D][4];
#pragma unroll
        for (int d = 0; d < D; d++) load_block(piece, b + d < last ? b + d : last, R[d]);
        for (;;) {
#pragma unroll
            for (int d = 0; d < D; d++) {
                bswap_block(R[d], w);
                load_block(piece, b + D < last ? b + D : last, R[d]);
                compress_full(h, w);
                if (++b >= g.fast_end) goto raw_done;
            }
        }
    }
raw_done:
    for (; b < g.end; b++) {
        build_tail_block(piece, len, b, w);
        uint32_t r[5];
        tv_sha1_full(h, r, w, TV_K0, TV_K1, TV_K2, TV_K3);
        if (b < nb) {
#pragma unroll
            for (int i = 0; i < 5; i++) h[i] += r[i];
        }
    }
    finish<HASH>(p, writer, jj, j0, h, last_grp);
}

// TV_LANE_PAD (A/B knob): 64-byte-align the kernel's first instructions, then TV_LANE_PAD 4-byte s_nops, which
// moves the raw-block loop through the 16 word positions of a 64-byte line (tools/build_variants.py D_TV_LANE_PAD)
#define TV_STR2(x) #x
#define TV_STR(x) TV_STR2(x)
template <bool HASH, bool PAIRS>
__global__ __launch_bounds__(256) void tv_lane_kernel(TvPieces p) {
#ifdef TV_LANE_PAD
    asm volatile(".p2align 6\n.rept " TV_STR(TV_LANE_PAD) "\ns_nop 0\n.endr\n" ::: "memory");
#endif
    ClockStamp clk;
    clk.start(p);
    lane_group<HASH, PAIRS>(p, blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    clk.end(p);
}

// ------------------------------------------------------------------------------------------
// split kernel: wave 0 = rounds (80 rounds per block from LDS), wave 1 = helper (loads +
// message schedule into a 3 x 20 KiB LDS ring, two blocks ahead).  One barrier per block.
// ------------------------------------------------------------------------------------------
namespace {

constexpr int kRingWords = 80 * 64;  // one buffer: [20 quads][64 lanes][4 words]
// K+W buffers per pair.  The helper runs TWO blocks ahead (block j lives in buffer j % 3), so the rounds
// wave can keep its 15 LDS reads in flight across block boundaries (tools/gen_sha1_asm.py
// gen_rounds_block) instead of restarting them, and an LDS latency, at every block.
constexpr uint32_t kBufs = TV_SHA1_LDS_BUFS;
constexpr uint32_t kAhead = TV_SHA1_HELPER_AHEAD;

__device__ __forceinline__ void lds_barrier() {
    // LDS writes of this wave complete, then the workgroup barrier.  Deliberately NOT
    // __syncthreads(): the helper's global prefetch loads must stay in flight across it.
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#if TV_STAMPS
// Diagnostic builds (tools/split_stamps.py; generator TV_GEN_STAMP=1 + -DTV_STAMPS=1): each split wave's asm loop
// time and the cycles its in-loop barriers (and, TV_SHA1_STAMP 2, the helper's vmcnt / lgkmcnt waits) took, per
// workgroup and wave, after the clock probe's 4 words: clock[4 + 8 (4 wg + wave) ..] = {loop cycles, barrier
// cycles, loop blocks, 1, vmcnt-wait cycles, lgkmcnt-wait cycles, 0, 0} (lane 0, vector stores).
static_assert(TV_SHA1_STAMP, "TV_STAMPS needs the generator's TV_GEN_STAMP header");
constexpr uint32_t kStampGroups = 65536;
struct LoopStamp {
    uint32_t bar = 0, vm = 0, lg = 0;
    uint64_t t0 = 0;
    __device__ __forceinline__ void start() { t0 = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void end(const TvPieces& p, uint32_t wave, uint32_t blocks) const {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (p.clock && blockIdx.x < kStampGroups && (threadIdx.x & 63u) == 0) {
            uint64_t* q = p.clock + 4 + 8 * (4 * (uint64_t)blockIdx.x + wave);
            reinterpret_cast<ulonglong2*>(q)[0] = make_ulonglong2(t1 - t0, bar);
            reinterpret_cast<ulonglong2*>(q)[1] = make_ulonglong2(blocks, 1);
            reinterpret_cast<ulonglong2*>(q)[2] = make_ulonglong2(vm, lg);
        }
    }
};
#endif

}  // namespace

__device__ __forceinline__ bool avail_bit(const uint64_t* a, uint32_t i) {
    // MSB-first bitfield bytes held in little-endian 64-bit words
    return (a[i >> 6] >> (((i >> 3) & 7) * 8 + (7 - (i & 7)))) & 1;
}

// LIST = incremental verify (tv_verify_list): lane j verifies shard piece idx[j]; one pair per
// workgroup, geometry from the pair's ballots (the short last piece may sit in any lane; the
// helper and rounds waves see the same 64 pieces, so their ballots agree).
// Workgroup-group wgi of a launch (PAIRS x {rounds, helper} waves, 64*PAIRS pieces), K+W ring in `ring`.
// The rounds wave calls before_state() (wave-uniform; false = give up) just before it reads its chaining
// state: the work-queue kernel waits there for the group's previous segment.
template <bool HASH, int PAIRS, bool LIST, typename BeforeState>
__device__ __forceinline__ void split_group(const TvPieces& p, uint32_t wgi, uint4* ring, BeforeState before_state) {
    // PAIRS x {rounds, helper} waves; 64*PAIRS pieces.  A workgroup's waves go to distinct SIMDs, so
    // with <= 1 workgroup per CU no rounds wave shares its SIMD.  Each pair has its own 3 x 20 KiB
    // K+W ring; the barrier is workgroup-wide, so both pairs run the same (workgroup) block range.
    static_assert(!LIST || PAIRS == 1, "list mode runs one pair per workgroup");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t pair = wave % PAIRS;
    const uint32_t role = wave / PAIRS;        // 0 = rounds, 1 = helper
    // main workgroups cover [0, n_main); a short last piece (n_main < n) gets one workgroup after
    // them, whose every lane (and pair) hashes it, so no main group runs its short tail.  List mode
    // has no last group (the host puts the last piece's entries in waves of their own).
    const uint32_t span = 64u * PAIRS;
    const uint32_t nlim = LIST ? p.n : p.n_main;
    const bool last_grp = !LIST && wgi >= (nlim + span - 1) / span;
    const uint32_t wg0 = last_grp ? p.last_idx : wgi * span;
    const uint32_t j0 = last_grp ? p.last_idx : wg0 + pair * 64u;
    const uint32_t j = last_grp ? p.last_idx : j0 + lane;
    const uint32_t jl = last_grp ? p.last_idx : (j < nlim ? j : nlim - 1);
    const uint32_t jj = LIST ? p.idx[jl] : jl;
    const bool is_last = jj == p.last_idx;
    const WaveGeom g = LIST ? wave_geom_flags(p, __ballot(is_last) != 0, __ballot(!is_last) == 0)
                            : last_grp ? wave_geom_flags(p, true, true) : wave_geom(p, wg0, span);
    const uint64_t len = lane_len(p, jj);
    const uint32_t nb = (uint32_t)nblocks(len);
    // (list mode over a slot pool: the entry's bytes sit in payload row rows[jl], TV_OPT_LIST_SLOTS)
    const uint32_t row = (LIST && p.rows) ? p.rows[jl] : jj;
    const uint8_t* piece = p.data + (uint64_t)row * p.stride - p.data_off;
    const uint32_t b0 = g.fast_begin, end = g.end, fast_end = g.fast_end;
    uint4* const pring = ring + pair * kBufs * (kRingWords / 4);

    if (role != 0) {
        // ---------------- helper wave ----------------
        // Block j of the launch goes to buffer j % 3, and the helper's barrier k follows its write of
        // block k + 1: it runs two blocks ahead.  Raw blocks [b0, fast_end): one asm loop (loads 2 blocks
        // ahead into registers the compiler never allocates, schedule, K+W -> LDS, a barrier after every
        // block but the first).  Then the 1-2 padded tail blocks and one spare block past `end` that the
        // rounds wave never consumes, in C++, and the barrier that matches the rounds wave's last one
        // (both waves execute end - b0 + 1 barriers).
        const uint32_t lds_lane = (uint32_t)(uintptr_t)(void*)pring + lane * 16u;
        uint32_t b = b0;
        if (fast_end > b0) {
#if TV_STAMPS
            LoopStamp st;
            st.start();
#if TV_SHA1_STAMP >= 2
            tv_sha1_helper_loop(piece + (uint64_t)b0 * 64, fast_end - b0, lds_lane, st.bar, st.vm, st.lg,
                                TV_K0, TV_K1, TV_K2, TV_K3);
#else
            tv_sha1_helper_loop(piece + (uint64_t)b0 * 64, fast_end - b0, lds_lane, st.bar, TV_K0, TV_K1, TV_K2, TV_K3);
#endif
            st.end(p, wave, fast_end - b0);
#else
            tv_sha1_helper_loop(piece + (uint64_t)b0 * 64, fast_end - b0, lds_lane, TV_K0, TV_K1, TV_K2, TV_K3);
#endif
            b = fast_end;
        }
        for (; b <= end; b++) {
            uint32_t w[16];
            build_tail_block(piece, len, b, w);
#pragma unroll
            for (int i = 0; i < 16; i++) w[i] = bswap32(w[i]);  // the schedule block byte-swaps
            tv_sha1_schedule_lds(w, lds_lane + ((b - b0) % kBufs) * (kRingWords * 4u), TV_K0, TV_K1, TV_K2, TV_K3);
            if (b - b0 + 1 >= kAhead) lds_barrier();
        }
        for (uint32_t k = 1; k < kAhead; k++) lds_barrier();
        return;
    }

    // ---------------- rounds wave ----------------
    uint32_t h[5];
    const bool go = before_state();   // (the helper waits at its first barrier meanwhile)
    if (LIST) sha1_iv(h);
    else if (go) start_state(p, jj, h);
    else sha1_iv(h);                  // abandoned (watchdog): the bits stay 0
    const uint32_t ring_base = (uint32_t)(uintptr_t)(void*)pring + lane * 16u;
    const uint32_t nb_min = g.nb_min;
    lds_barrier();
    uint32_t b = b0;
    // blocks where every lane of the wave updates: one asm loop (rounds, h += r, barrier)
    const uint32_t full_end = end < nb_min ? end : nb_min;
    if (b < full_end) {
#if TV_STAMPS
        LoopStamp st;
        st.start();
        tv_sha1_rounds_loop(h, ring_base, full_end - b, st.bar, TV_K0, TV_K1, TV_K2, TV_K3);
        st.end(p, wave, full_end - b);
#else
        tv_sha1_rounds_loop(h, ring_base, full_end - b, TV_K0, TV_K1, TV_K2, TV_K3);
#endif
        b = full_end;
    }
    // the short last piece's wave: lanes past their final block keep their digest
    for (; b < end; b++) {
        uint32_t r[5];
        tv_sha1_lds(h, r, ring_base + ((b - b0) % kBufs) * (kRingWords * 4u), TV_K0, TV_K1, TV_K2, TV_K3);
        if (b < nb) {
#pragma unroll
            for (int i = 0; i < 5; i++) h[i] += r[i];
        }
        lds_barrier();
    }
    if (LIST) {
        if (j < p.n) {
            bool ok = p.avail64 ? avail_bit(p.avail64, jj) : true;
#pragma unroll
            for (int k = 0; k < 5; k++) ok &= (h[k] == p.digests[(uint64_t)k * p.dcount + jj]);
            p.out_bytes[j] = ok ? 1 : 0;
        }
        return;
    }
    finish<HASH>(p, go && (last_grp ? (lane == 0 && pair == 0) : j < p.n_main), jj, j0, h, last_grp);
}

template <bool HASH, int PAIRS, bool LIST = false>
__global__ __launch_bounds__(128 * PAIRS) void tv_split_kernel(TvPieces p) {
    __shared__ __attribute__((aligned(16))) uint4 ring[kBufs * PAIRS * kRingWords / 4];
    ClockStamp clk;
    clk.start(p);
    split_group<HASH, PAIRS, LIST>(p, blockIdx.x, ring, [] { return true; });
    clk.end(p);   // (the rounds wave, wave 0, returns from split_group last)
}

// ------------------------------------------------------------------------------------------
// twin kernel: the split kernel with TWO lanes per piece in every wave.  A workgroup is rounds waves 0, 1
// and helper waves 2, 3 over 64 pieces; in each wave lane 2i + b runs piece 32(wave & 1) + i and owns its
// schedule words of parity b (tools/gen_sha1_asm.py gen_twin / gen_helper2).  Rounds: both lanes of a pair
// run the same rounds; lane b reads only its own K+W words and each round's `e + KW` add takes KW from lane
// t % 2 of the pair through DPP: 10 ds_read_b128 per block instead of 20, serial stream 405 VALU + 10 LDS
// + 2 waits.  Helper: 192 VALU + 10 ds_write_b128 per block (W[32..79] from the parity-closed recurrence
// W[t] = rotl2(W[t-6] ^ W[t-16] ^ W[t-28] ^ W[t-32])), half a split helper's stream.  K+W ring: 3 x 20 KiB,
// the helpers two blocks ahead, one 4-wave barrier per block.  Four waves per 64 pieces fill the SIMDs up
// to 16,384 pieces (cfg2: 256 workgroups, one per CU).
// ------------------------------------------------------------------------------------------
namespace {

// Final step of a twin rounds wave (32 pieces, lane 2i + b = piece j0w + i): as finish(), with the
// bitfield bits of the even lanes.
template <bool HASH>
__device__ __forceinline__ void finish_twin(const TvPieces& p, bool writer, uint32_t jj, uint32_t j0w,
                                            const uint32_t h[5], bool last_grp) {
    if (!p.finalize || HASH) {
        finish<HASH>(p, writer, jj, j0w, h, last_grp);
        return;
    }
    bool ok = writer;
#pragma unroll
    for (int k = 0; k < 5; k++) ok &= (h[k] == p.digests[(uint64_t)k * p.dcount + jj]);
    const uint64_t mask = __ballot(ok);
    if ((threadIdx.x & 63) == 0) {
        uint64_t bits;
        uint32_t w;
        if (last_grp) {
            w = jj >> 6;
            bits = (mask & 1) ? 1ull << (((jj >> 3) & 7) * 8 + 7 - (jj & 7)) : 0;
        } else {
            uint64_t x = mask & 0x5555555555555555ull;          // even lanes -> bits 0..31
            x = (x | (x >> 1)) & 0x3333333333333333ull;
            x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
            x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
            x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
            x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
            w = j0w >> 6;
            bits = __builtin_bswap64(__builtin_bitreverse64(x << (j0w & 63)));
        }
        if (p.avail64) bits &= p.avail64[w];
        if (bits) atomicOr(reinterpret_cast<unsigned long long*>(p.out64 + w), (unsigned long long)bits);
    }
}

}  // namespace

// Workgroup shapes (wave -> role and 32-piece half; the hardware puts a workgroup's waves on SIMDs in the
// cyclic order 0 -> 2 -> 1 -> 3 from a varying start, MI355X_MICROARCH.md section LDS):
//   1: 2 waves {rounds, helper} over 32 pieces, two workgroups per CU (the auto shape)
//   2: 4 waves, rounds {0, 1}, helpers {2, 3} over 64 pieces      3: rounds {0, 2}, helpers {1, 3}
//   4: 4 waves over 32 pieces, rounds 0, helper 2, waves 1 and 3 idle at the barriers   5: helper 1, idle 2, 3
// (shapes 3-5 are SIMD-placement probes: tools/twin_occupancy_probe.py)
constexpr int kTwinRole[6][4] = {{0, 0, 0, 0}, {0, 1, 2, 2}, {0, 0, 1, 1}, {0, 1, 0, 1}, {0, 2, 1, 2}, {0, 1, 2, 2}};
constexpr int kTwinHalf[6][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 1, 0, 1}, {0, 0, 1, 1}, {0, 0, 0, 0}, {0, 0, 0, 0}};
constexpr int kTwinWaves[6] = {0, 2, 4, 4, 4, 4};
constexpr int kTwinPairs[6] = {0, 1, 2, 2, 1, 1};

// LIST = incremental verify (tv_verify_list): pair i of a wave verifies shard piece idx[j]; geometry from the
// wave's ballots (the rounds and helper waves of a half see the same 32 pieces, so their ballots agree); the
// host puts the short last piece's entries in 64-entry groups of their own.
template <bool HASH, int SHAPE, bool LIST = false>
__global__ __launch_bounds__(64 * kTwinWaves[SHAPE]) void tv_twin_kernel(TvPieces p) {
    __shared__ __attribute__((aligned(16))) uint4 ring[kBufs * kRingWords / 4];
    constexpr uint32_t span = 32u * kTwinPairs[SHAPE];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int role = kTwinRole[SHAPE][wave];                  // 0 rounds, 1 helper, 2 idle
    const uint32_t half = kTwinHalf[SHAPE][wave];             // pieces 32*half .. +31
    // main workgroups cover [0, n_main); a short last piece gets one workgroup after them (every lane)
    const uint32_t nlim = LIST ? p.n : p.n_main;
    // companions (blockIdx past the real grid, TV_OPT_TWIN_FILL): re-hash main workgroup (blockIdx - real) % main
    const uint32_t nmain_wgs = (nlim + span - 1) / span;
    const uint32_t real_wgs = nmain_wgs + (!LIST && p.n_main < p.n ? 1u : 0u);
    const bool companion = blockIdx.x >= real_wgs;
    const uint32_t wgi = companion ? (blockIdx.x - real_wgs) % nmain_wgs : blockIdx.x;
    const bool last_grp = !LIST && wgi >= nmain_wgs;
    const uint32_t wg0 = last_grp ? p.last_idx : wgi * span;
    // a companion keeps the instruction stream of the workgroup it copies but, unless fill_all, points every
    // lane at that workgroup's first piece: the same loads, one piece's bytes instead of 32 pieces'
    const uint32_t j = last_grp ? p.last_idx : (companion && !p.fill_all ? wg0 : wg0 + half * 32u + (lane >> 1));
    const uint32_t jl = last_grp ? p.last_idx : (j < nlim ? j : nlim - 1);
    const uint32_t jj = LIST ? p.idx[jl] : jl;
    const bool is_last = jj == p.last_idx;
    const WaveGeom g = LIST ? wave_geom_flags(p, __ballot(is_last) != 0, __ballot(!is_last) == 0)
                            : last_grp ? wave_geom_flags(p, true, true) : wave_geom(p, wg0, span);
    const uint64_t len = lane_len(p, jj);
    const uint32_t nb = (uint32_t)nblocks(len);
    const uint32_t row = (LIST && p.rows) ? p.rows[jl] : jj;   // (slot pool: TV_OPT_LIST_SLOTS)
    const uint8_t* piece = p.data + (uint64_t)row * p.stride - p.data_off;
    const uint32_t b0 = g.fast_begin, end = g.end, fast_end = g.fast_end;
    const uint32_t lds_lane = (uint32_t)(uintptr_t)(void*)ring + half * 1024u + lane * 16u;
    ClockStamp clk;
    clk.start(p);

    if (role == 2) {   // idle wave: the same number of barriers as the others (end - b0 + 1)
        for (uint32_t b = b0; b <= end; b++) lds_barrier();
        return;
    }
    if (role == 1) {
        // ---------------- helper waves (as split_group's helper, twin layout) ----------------
        const uint32_t psel = (lane & 1u) ? 0x07060504u : 0x03020100u;
        uint32_t b = b0;
        if (fast_end > b0) {
#if TV_STAMPS
            LoopStamp st;
            st.start();
#if TV_SHA1_STAMP >= 2
            tv_sha1_twin_helper_loop(piece + (uint64_t)b0 * 64, fast_end - b0, lds_lane, psel, st.bar, st.vm, st.lg,
                                     TV_K0, TV_K1, TV_K2, TV_K3);
#else
            tv_sha1_twin_helper_loop(piece + (uint64_t)b0 * 64, fast_end - b0, lds_lane, psel, st.bar,
                                     TV_K0, TV_K1, TV_K2, TV_K3);
#endif
            st.end(p, wave, fast_end - b0);
#else
            tv_sha1_twin_helper_loop(piece + (uint64_t)b0 * 64, fast_end - b0, lds_lane, psel, TV_K0, TV_K1, TV_K2, TV_K3);
#endif
            b = fast_end;
        }
        for (; b <= end; b++) {
            uint32_t w[16];
            build_tail_block(piece, len, b, w);
#pragma unroll
            for (int i = 0; i < 16; i++) w[i] = bswap32(w[i]);  // the schedule block byte-swaps
            tv_sha1_twin_schedule_lds(w, lds_lane + ((b - b0) % kBufs) * (kRingWords * 4u), psel, TV_K0, TV_K1, TV_K2, TV_K3);
            if (b - b0 + 1 >= kAhead) lds_barrier();
        }
        for (uint32_t k = 1; k < kAhead; k++) lds_barrier();
        return;
    }

    // ---------------- rounds waves ----------------
    uint32_t h[5];
    if (LIST) sha1_iv(h);
    else start_state(p, jj, h);
    const uint32_t ring_base = lds_lane;
    lds_barrier();
    uint32_t b = b0;
    const uint32_t full_end = end < g.nb_min ? end : g.nb_min;
    if (b < full_end) {
#if TV_STAMPS
        LoopStamp st;
        st.start();
        tv_sha1_twin_rounds_loop(h, ring_base, full_end - b, st.bar);
        st.end(p, wave, full_end - b);
#else
        tv_sha1_twin_rounds_loop(h, ring_base, full_end - b);
#endif
        b = full_end;
    }
    // the short last piece's workgroup: lanes past their final block keep their digest (both lanes of a
    // pair hold the same piece, so the DPP partner is always in step)
    for (; b < end; b++) {
        uint32_t r[5];
        tv_sha1_twin_lds(h, r, ring_base + ((b - b0) % kBufs) * (kRingWords * 4u));
        if (b < nb) {
#pragma unroll
            for (int i = 0; i < 5; i++) h[i] += r[i];
        }
        lds_barrier();
    }
    clk.end(p);              // (wave 0 is a rounds wave in every shape)
    if (companion) return;   // its digests duplicate a main workgroup's: nothing to write
    if (LIST) {
        if (j < p.n && (lane & 1u) == 0) {
            bool ok = p.avail64 ? avail_bit(p.avail64, jj) : true;
#pragma unroll
            for (int k = 0; k < 5; k++) ok &= (h[k] == p.digests[(uint64_t)k * p.dcount + jj]);
            p.out_bytes[j] = ok ? 1 : 0;
        }
        return;
    }
    const bool writer = last_grp ? (wave == 0 && lane == 0) : ((lane & 1u) == 0 && j < p.n_main);
    finish_twin<HASH>(p, writer, jj, wg0 + half * 32u, h, last_grp);
}

// ------------------------------------------------------------------------------------------
// list kernel (incremental verify): lane j verifies shard piece idx[j]; same compression path as
// the lane kernel, geometry from wave ballots (the short last piece may sit in any lane).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tv_list_kernel(TvPieces p) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t j0 = blockIdx.x * 256u + wave * 64u;
    if (j0 >= p.n) return;
    const uint32_t j = j0 + (threadIdx.x & 63u);
    const uint32_t jl = j < p.n ? j : p.n - 1;
    const uint32_t jj = p.idx[jl];
    const bool is_last = jj == p.last_idx;
    const WaveGeom g = wave_geom_flags(p, __ballot(is_last) != 0, __ballot(!is_last) == 0);
    const uint64_t len = is_last ? p.last_len : p.L;
    const uint32_t nb = (uint32_t)nblocks(len);
    const uint8_t* piece = p.data + (uint64_t)(p.rows ? p.rows[jl] : jj) * p.stride;   // (slot pool)
    uint32_t h[5];
    sha1_iv(h);
    uint32_t b = 0, w[16];
    if (b < g.fast_end) {
        const uint32_t last = g.fast_end - 1;
        uint4 A[4], B[4];
        load_block(piece, 0, A);
        load_block(piece, 1 < last ? 1 : last, B);
        for (;;) {
            bswap_block(A, w);
            load_block(piece, b + 2 < last ? b + 2 : last, A);
            compress_full(h, w);
            if (++b >= g.fast_end) break;
            bswap_block(B, w);
            load_block(piece, b + 2 < last ? b + 2 : last, B);
            compress_full(h, w);
            if (++b >= g.fast_end) break;
        }
    }
    for (; b < g.end; b++) {
        build_tail_block(piece, len, b, w);
        uint32_t r[5];
        tv_sha1_full(h, r, w, TV_K0, TV_K1, TV_K2, TV_K3);
        if (b < nb) {
#pragma unroll
            for (int i = 0; i < 5; i++) h[i] += r[i];
        }
    }
    if (j < p.n) {
        bool ok = p.avail64 ? avail_bit(p.avail64, jj) : true;
#pragma unroll
        for (int k = 0; k < 5; k++) ok &= (h[k] == p.digests[(uint64_t)k * p.dcount + jj]);
        p.out_bytes[j] = ok ? 1 : 0;
    }
}

// ------------------------------------------------------------------------------------------
// synthetic payload fill: byte at linear offset o = byte (o & 7) of splitmix64(seed, o >> 3).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// L % 8 == 0: whole 8-byte words.  Piece j of the launch = global piece first + j.
__global__ __launch_bounds__(256) void tv_fill_words_kernel(uint8_t* payload, uint64_t stride, uint64_t first,
                                                            uint32_t n, uint64_t L, uint64_t seed) {
    const uint64_t wpp = L / 8;
    const uint64_t total = wpp * n;
    for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256ull) {
        const uint64_t j = g / wpp, k = g - j * wpp;
        const uint64_t o = (first + j) * L + 8 * k;
        *reinterpret_cast<uint64_t*>(payload + j * stride + 8 * k) = splitmix64(seed, o >> 3);
    }
}

__global__ __launch_bounds__(256) void tv_fill_bytes_kernel(uint8_t* payload, uint64_t stride, uint64_t first,
                                                            uint32_t n, uint64_t L, uint64_t seed) {
    const uint64_t total = L * n;
    for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256ull) {
        const uint64_t j = g / L, k = g - j * L;
        const uint64_t o = (first + j) * L + k;
        payload[j * stride + k] = (uint8_t)(splitmix64(seed, o >> 3) >> (8 * (o & 7)));
    }
}

// ------------------------------------------------------------------------------------------
// windowed layouts (tv_core.hip): the windows are hashed (HASH kernels into the shard's digest rows) as they
// fill, and tv_verify compares the whole shard at the end -- 40 B read per piece, one word written per 64.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tv_compare_kernel(const uint32_t* hash, const uint32_t* digests,
                                                         uint32_t dcount, uint32_t n, const uint64_t* avail64,
                                                         uint64_t* out64) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    bool ok = j < n;
    if (ok) {
#pragma unroll
        for (int k = 0; k < 5; k++) ok &= hash[(uint64_t)k * dcount + j] == digests[(uint64_t)k * dcount + j];
    }
    const uint64_t mask = __ballot(ok);
    if ((threadIdx.x & 63u) == 0) {   // lane 0 of the wave: pieces j .. j + 63, word j >> 6
        uint64_t bits = __builtin_bswap64(__builtin_bitreverse64(mask));   // ballot bit l -> MSB-first bytes
        if (avail64) bits &= avail64[j >> 6];
        out64[j >> 6] = bits;
    }
}

// ------------------------------------------------------------------------------------------
// host-side launchers (called by tv_core.hip, tv_stream.hip, tv_verify.hip)
// ------------------------------------------------------------------------------------------
hipError_t tv_launch_verify(const TvPieces& p, int kernel, bool hash, hipStream_t s, int split_pairs,
                            uint32_t* workgroups) {
    if (workgroups) *workgroups = 0;
    if (p.n == 0) return hipSuccess;
    if (kernel == TV_KERNEL_SPLIT) {
        // one pair per workgroup: with its 60 KiB LDS ring at most two workgroups share a CU, and up to
        // 32,768 pieces every rounds wave still gets a SIMD of its own; 1 pair beats 2 pairs (one 4-wave
        // barrier couples more jitter) at every piece count up to there, by 1.7-3 % (profiles/r02/sweep_3buf.log)
        const int pairs = (split_pairs == 1 || split_pairs == 2) ? split_pairs : 1;
        const unsigned grid = (p.n_main + 64 * pairs - 1) / (64 * pairs) + (p.n_main < p.n ? 1 : 0);
        if (workgroups) *workgroups = grid;
        if (pairs == 1) {
            if (hash) hipLaunchKernelGGL((tv_split_kernel<true, 1>), dim3(grid), dim3(128), 0, s, p);
            else hipLaunchKernelGGL((tv_split_kernel<false, 1>), dim3(grid), dim3(128), 0, s, p);
        } else {
            if (hash) hipLaunchKernelGGL((tv_split_kernel<true, 2>), dim3(grid), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((tv_split_kernel<false, 2>), dim3(grid), dim3(256), 0, s, p);
        }
    } else if (kernel == TV_KERNEL_TWIN) {
        // split_pairs: (rounds, helper) pairs per workgroup: 1 (auto) = 2-wave workgroups over 32 pieces, two
        // per CU; 2 = the 4-wave workgroup over 64 pieces, whose 4-wave barrier couples more jitter (cfg2
        // 1,419 vs 1,358 GB/s, profiles/r02/sweep_twin.log)
        // (3-5: SIMD-placement probe shapes, see tv_twin_kernel)
        const int shape = split_pairs >= 2 && split_pairs <= 5 ? split_pairs : 1;
        const unsigned span = 32u * kTwinPairs[shape];
        const unsigned real = (p.n_main + span - 1) / span + (p.n_main < p.n ? 1 : 0);
        const unsigned grid = (p.fill_to > real && p.n_main > 0) ? p.fill_to : real;
        if (workgroups) *workgroups = grid;
        const dim3 blk(64 * kTwinWaves[shape]);
#define TV_TWIN_LAUNCH(S)                                                              \
    if (hash) hipLaunchKernelGGL((tv_twin_kernel<true, S>), dim3(grid), blk, 0, s, p); \
    else hipLaunchKernelGGL((tv_twin_kernel<false, S>), dim3(grid), blk, 0, s, p);
        switch (shape) {
            case 2: TV_TWIN_LAUNCH(2) break;
            case 3: TV_TWIN_LAUNCH(3) break;
            case 4: TV_TWIN_LAUNCH(4) break;
            case 5: TV_TWIN_LAUNCH(5) break;
            default: TV_TWIN_LAUNCH(1) break;
        }
#undef TV_TWIN_LAUNCH
    } else {
        const unsigned waves = (p.n_main + 63) / 64 + (p.n_main < p.n ? 1 : 0);
        const unsigned grid = (waves + 3) / 4;
        if (workgroups) *workgroups = grid;
        if (p.lane_pairs) {
            if (hash) hipLaunchKernelGGL((tv_lane_kernel<true, true>), dim3(grid), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((tv_lane_kernel<false, true>), dim3(grid), dim3(256), 0, s, p);
        } else {
            if (hash) hipLaunchKernelGGL((tv_lane_kernel<true, false>), dim3(grid), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((tv_lane_kernel<false, false>), dim3(grid), dim3(256), 0, s, p);
        }
    }
    return hipGetLastError();
}

hipError_t tv_launch_verify_list(const TvPieces& p, int kernel, hipStream_t s, uint32_t* workgroups) {
    if (workgroups) *workgroups = 0;
    if (p.n == 0) return hipSuccess;
    unsigned grid;
    if (kernel == TV_KERNEL_TWIN) {
        const unsigned real = (p.n + 31) / 32;
        grid = p.fill_to > real ? p.fill_to : real;
        hipLaunchKernelGGL((tv_twin_kernel<false, 1, true>), dim3(grid), dim3(128), 0, s, p);
    } else if (kernel == TV_KERNEL_SPLIT) {
        grid = (p.n + 63) / 64;
        hipLaunchKernelGGL((tv_split_kernel<false, 1, true>), dim3(grid), dim3(128), 0, s, p);
    } else {
        grid = (p.n + 255) / 256;
        hipLaunchKernelGGL(tv_list_kernel, dim3(grid), dim3(256), 0, s, p);
    }
    if (workgroups) *workgroups = grid;
    return hipGetLastError();
}

hipError_t tv_launch_fill(uint8_t* payload, uint64_t stride, uint64_t first, uint32_t n, uint64_t L,
                          uint64_t seed, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = 256 * 32;
    if (L % 8 == 0) hipLaunchKernelGGL(tv_fill_words_kernel, dim3(grid), dim3(256), 0, s, payload, stride, first, n, L, seed);
    else hipLaunchKernelGGL(tv_fill_bytes_kernel, dim3(grid), dim3(256), 0, s, payload, stride, first, n, L, seed);
    return hipGetLastError();
}

hipError_t tv_launch_compare(const uint32_t* hash, const uint32_t* digests, uint32_t dcount, uint32_t n,
                             const uint64_t* avail64, uint64_t* out64, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(tv_compare_kernel, dim3((n + 255) / 256), dim3(256), 0, s, hash, digests, dcount, n, avail64, out64);
    return hipGetLastError();
}
