// tv_internal.h -- shared between the kernels (tv_kernels.hip) and the C ABI (tv_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TV_KERNEL_AUTO 0
#define TV_KERNEL_LANE 1
#define TV_KERNEL_SPLIT 2
#define TV_KERNEL_MIX 3     // work queue: split pairs + lane waves share 64-piece groups segment by segment
#define TV_KERNEL_TWIN 4    // split with two lanes per piece in the rounds waves (half the K+W reads per block)

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
};

// Work queue of the MIX launch (tv_launch_mix): a FIFO of ready 64-piece groups.  A unit is segment s
// (blocks [s * seg_blocks, (s + 1) * seg_blocks); the last one runs to the end and finalises) of group g;
// entries are (lap tag << 32 | s << 16 | g), so groups and segs are < 65,536.
struct TvQueue {
    uint32_t* head;      // pop tickets   (head, tail, error: zeroed before the launch)
    uint32_t* tail;      // push tickets
    uint32_t* error;     // nonzero: a worker's wait exceeded the watchdog; the launch's output is invalid
    uint64_t* slots;     // [ring] entries (zeroed before the launch)
    uint32_t ring;       // >= groups
    uint32_t groups, segs, seg_blocks, units;  // units = groups * segs
    uint64_t* trace;     // diagnostics (tools/mix_probe.cpp), null in the library: per unit (s * groups + g)
                         // {pop, start, end} s_memrealtime ticks and the worker id
};

// Worker shape of a MIX launch: pair_wgs split-pair workgroups declaring pair_lds_bufs (3 or 5) K+W
// buffers of LDS, lane_wgs lane workgroups of lane_waves_per_wg (1..4) waves each, lane_lds bytes of
// (unused) dynamic LDS per lane workgroup.
struct TvMixShape {
    unsigned pair_wgs, pair_lds_bufs, lane_wgs, lane_waves_per_wg, lane_lds;
};

hipError_t tv_launch_verify(const TvPieces& p, int kernel, bool hash, hipStream_t s, int split_pairs = 0);
// The MIX launch: the pair workers on s_pairs and the lane workers on s_lanes, concurrently, over the
// queue q (the short last piece, if any, is a group of its own like in tv_launch_verify).
hipError_t tv_launch_mix(const TvPieces& p, const TvQueue& q, bool hash, hipStream_t s_pairs, hipStream_t s_lanes,
                         const TvMixShape& m);
hipError_t tv_launch_verify_list(const TvPieces& p, int kernel, hipStream_t s);
hipError_t tv_launch_fill(uint8_t* payload, uint64_t stride, uint64_t first, uint32_t n, uint64_t L,
                          uint64_t seed, hipStream_t s);
