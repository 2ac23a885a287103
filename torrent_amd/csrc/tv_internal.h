// tv_internal.h -- shared between the kernels (tv_kernels.hip) and the C ABI (tv_core.hip, tv_context.hip, ...: see tv_ctx.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TV_KERNEL_AUTO 0
#define TV_KERNEL_LANE 1
#define TV_KERNEL_SPLIT 2
// (3 was MIX, a work queue over split pairs and lane waves: measured 8.6 % slower than lane where lane is
//  chosen, removed in round 3; the value stays unused)
#define TV_KERNEL_TWIN 4    // split with two lanes per piece in the rounds waves (half the K+W reads per block)

#ifndef TV_STAMPS
#define TV_STAMPS 0   // 1: diagnostic split-kernel loop stamps (tools/split_stamps.py), never the shipped library
#endif
// words of the device clock buffer (TV_OPT_CLOCK_PROBE): the probe's 4, plus in TV_STAMPS builds 8 per wave of up
// to 4 waves in each of 65,536 workgroups
constexpr size_t kClockWords = 4 + (TV_STAMPS ? 8 * 4 * 65536 : 0);

// One launch over a contiguous run of n pieces.  Piece j's byte k (piece-relative) is at
// data + j*stride + k - data_off.  Blocks [blk_begin, min(blk_end, nb_j)) are processed.
struct TvPieces {
    const uint8_t* data;
    uint64_t stride;
    uint64_t data_off;
    uint64_t L;              // piece length of every piece except last_idx
    uint64_t last_len;       // length of piece last_idx
    uint64_t blk_begin;
    uint64_t blk_end;        // UINT64_MAX = through the end of every piece
    uint32_t n;
    uint32_t n_main;         // main groups cover pieces [0, n_main); n_main = n - 1 when the short last
                             // piece (last_len < L) gets a group of its own, else n (list mode: n)
    uint32_t last_idx;       // launch-local index of the torrent's last piece, 0xFFFFFFFF if absent
    uint32_t finalize;       // 1: compare / emit digests; 0: store chaining values to `state`
    uint32_t dcount;         // row stride of state / digests / out_digests (= shard piece count)
    uint32_t* state;         // [5][dcount] chaining values (read when blk_begin > 0, written when !finalize)
    const uint32_t* digests; // [5][dcount] expected digest words (big-endian values)
    const uint64_t* avail64; // MSB-first bitfield bytes over the shard (64-bit words); may be null
    uint64_t* out64;         // per 64 pieces, MSB-first bitfield bytes (sized to whole 256-piece groups)
    uint32_t* out_digests;   // hash mode: [5][dcount]
    const uint32_t* idx;     // list mode: lane j verifies shard piece idx[j] (data = base + idx*stride)
    uint8_t* out_bytes;      // list mode: out_bytes[j] = 1 iff piece idx[j] matches
    uint32_t fill_to;        // twin: launch this many workgroups in all (0 = the real grid only); the ones past
                             // the real grid are COMPANIONS that re-hash a main workgroup's pieces and discard
                             // the result (TV_OPT_TWIN_FILL)
    uint32_t fill_all;       // companions: 0 = every lane hashes the main workgroup's FIRST piece (the same
                             // instruction stream, 1/32 of the reads), 1 = its 32 pieces (TV_OPT_TWIN_FILL_READS)
    const uint32_t* rows;    // list mode with a slot pool (TV_OPT_LIST_SLOTS): entry j's bytes are payload row
                             // rows[j] (data + rows[j]*stride) while digests / length / availability stay those of
                             // piece idx[j]; null = row idx[j]
    uint64_t* clock;         // TV_OPT_CLOCK_PROBE: lane 0 of workgroup 0's (rounds) wave stores {shader clock counter,
                             // 100 MHz real-time counter} at its start and end here (4 words); null = off
    uint32_t lane_pairs;     // host-side choice for the lane kernel: 1 = the pair-load instantiation (a lane's two
                             // 64-B blocks of a 128-B line loaded back to back; >= 1 wave per SIMD), 0 = 3-deep ring
};

// workgroups (optional): set to the launch's grid size, companions included.
hipError_t tv_launch_verify(const TvPieces& p, int kernel, bool hash, hipStream_t s, int split_pairs = 0,
                            uint32_t* workgroups = nullptr);
hipError_t tv_launch_verify_list(const TvPieces& p, int kernel, hipStream_t s, uint32_t* workgroups = nullptr);
hipError_t tv_launch_fill(uint8_t* payload, uint64_t stride, uint64_t first, uint32_t n, uint64_t L,
                          uint64_t seed, hipStream_t s);
// Windowed layouts: bit j of out64 (MSB-first bytes in 64-bit words, as the verify kernels write it) = the
// digest hash[.][j] equals digests[.][j] ([5][dcount] SoA) and avail64 bit j (null: all); j < n, the rest 0.
hipError_t tv_launch_compare(const uint32_t* hash, const uint32_t* digests, uint32_t dcount, uint32_t n,
                             const uint64_t* avail64, uint64_t* out64, hipStream_t s);
