// tv_plan.h -- the resident payload's shape under a device budget (tv_set_layout), a stream's windows x columns under
// one (stream_geometry) and the file table's walk (walk_file_table), as plain host code with no HIP in it, so they are
// unit-tested on the CPU (tests/c/plan_test.cpp, tests/c/walk_main.cpp, tests/test_plan.py).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace tvi {

struct PayloadPlan {
    uint64_t bytes = 0;      // the allocation (0: none)
    bool win = false;        // windowed: `bufs` buffers of `win_n` pieces, `buf_bytes` each
    uint64_t win_n = 0;
    int bufs = 0;
    uint64_t buf_bytes = 0;
};

// Window buffers of a windowed layout by default (TV_OPT_WIN_BUFS = 0): window w + 1 stages while the two windows
// before it hash side by side, on the compute stream and one hash stream (a window's hash takes one piece's serial
// SHA-1 whatever its piece count, so under a small budget windows must hash side by side to keep staging busy).
// Three beat two and four at HIP's default 4 hardware queues: 0.5 GiB 28.3 / 22.2 / 26.5 GB/s, 1 GiB 51.6 / 38.5 /
// 45.2 (profiles/r06/window_bench_shipped_form.jsonl).
constexpr int kWinBufsDefault = 3;
constexpr int kWinBufsMax = 8;

// `count` pieces at `stride` bytes (+ `slack` after the last) under `budget` bytes: the whole shard when it fits,
// else `bufs` window buffers of W pieces (fewer buffers when the budget cannot hold one piece in each; never more
// than there are windows; W >= 1 even when one piece exceeds the budget; a multiple of 64 from 256 up, so each
// window is whole 64-piece waves).
inline PayloadPlan plan_payload(uint64_t count, uint64_t stride, uint64_t slack, uint64_t budget,
                                int bufs = kWinBufsDefault) {
    PayloadPlan p;
    if (count == 0) return p;
    p.bytes = count * stride + slack;
    if (p.bytes <= budget) return p;
    uint64_t B = (uint64_t)std::max(1, std::min(bufs, kWinBufsMax)), W = 0;
    for (; B > 1; B--) {
        W = budget / B > slack ? (budget / B - slack) / stride : 0;
        if (W) break;
    }
    if (B == 1) W = budget > slack ? (budget - slack) / stride : 0;
    W = std::max<uint64_t>(1, std::min(W, count));
    if (W >= 256) W = W / 64 * 64;
    B = std::max<uint64_t>(1, std::min(B, (count + W - 1) / W));
    p.win = true;
    p.win_n = W;
    p.bufs = (int)B;
    p.buf_bytes = W * stride + slack;
    p.bytes = B * p.buf_bytes;
    return p;
}

// Plan and allocate: try_alloc(plan, budget) -> 0 (the plan's bytes are held), 1 (out of memory), 2 (another
// failure).  Out of memory is retried with windows at half the budget while the request still shrinks and is
// above 64 MiB; a plan that cannot get smaller (a one-piece window of a piece larger than the memory left) is out of
// memory, not a retry forever.  Returns 0 (*out, *budget_out: what is held), 1 or 2; *failed_bytes:
// the last request that failed.
template <class TryAlloc>
int allocate_payload(uint64_t count, uint64_t stride, uint64_t slack, uint64_t budget, TryAlloc&& try_alloc,
                     PayloadPlan* out, uint64_t* budget_out, uint64_t* failed_bytes, int bufs = kWinBufsDefault) {
    uint64_t failed = UINT64_MAX;
    for (;;) {
        const PayloadPlan p = plan_payload(count, stride, slack, budget, bufs);
        const int r = try_alloc(p, budget);
        if (r == 0) {
            *out = p;
            *budget_out = budget;
            return 0;
        }
        *failed_bytes = p.bytes;
        if (r != 1 || p.bytes <= (64ull << 20) || p.bytes >= failed) return r;
        failed = p.bytes;
        budget = p.bytes / 2;  // windows of half the size
    }
}

// One segment of Storage.get's walk over a torrent's file table: `len` bytes of file `file` from byte `file_offset`
// are LINEAR bytes [linear, linear + len); len == 0 for the walk's zero-length segments.
struct TableSeg {
    uint64_t file, file_offset, linear, len;
};

// findAndDo's walk (storage.ts:98-137) over the files in order -- file k holds lengths[k] bytes and starts where the
// files before it end -- restricted to the LINEAR bytes [lo, hi) of a shard (lo a multiple of L): every segment with
// bytes there, and the zero-length segments fsStorage.get still opens (storage.ts:109-110,158): a file ending inside
// [lo, hi) that is empty or ends exactly where a piece starts.  The hosts' walks make the same list
// (torrent_amd/verify.py _files_shard over storage.py segment_arrays / zero_length_segments).  *reached: where the
// walk stopped (< hi: the files end before the shard does, and Storage.get returns null for a piece past their end).
// false (*bad = the file) when the lengths overflow 64-bit offsets.  tv_stage_file_table uses it;
// tests/c/walk_main.cpp runs it on the CPU.
inline bool walk_file_table(uint64_t n, const uint64_t* lengths, uint64_t lo, uint64_t hi, uint64_t L,
                            std::vector<TableSeg>* out, uint64_t* bad, uint64_t* reached) {
    uint64_t start = 0;
    for (uint64_t k = 0; k < n && start < hi; k++) {
        if (lengths[k] > UINT64_MAX - start) {
            *bad = k;
            return false;
        }
        const uint64_t end = start + lengths[k];
        const uint64_t a = std::max(lo, start), b = std::min(hi, end);
        if (b > a) out->push_back({k, a - start, a, b - a});
        if (end >= lo && end < hi && (lengths[k] == 0 || end % L == 0)) out->push_back({k, lengths[k], end, 0});
        start = end;
    }
    *reached = start;
    return true;
}

// ---- a stream's geometry under a device budget (tv_stream.hip: tv_stream_file_table, tv_verify_host) ----------------
//
// Windows of at least `min_win` pieces (a multiple of 64 unless the shard is smaller), each hashed column by column --
// enough pieces that a column hashes faster than it stages (2,048 pieces x 64 B per ~0.75 us block step: ~175 GB/s)
// -- and columns as wide as two chunk buffers within the budget allow, so each row is one long read or DMA row: 124 KiB
// at a 0.5 GiB budget and 1 MiB pieces where columns across all 16,384 pieces would be 16 KiB.  A multiple of 4 KiB
// from 4 KiB up (a cold file's rows are read O_DIRECT straight into the ring slot); where whole pieces fit, the
// windows grow to fill the budget.  Each chunk buffer is at most kStreamChunkMax: wider columns gained nothing and
// larger units overlap less (the first unit's copy and the last unit's kernel run alone): budgets of 2 GiB (1 GiB
// units) ran 44-49 GB/s against 52-55 at 0.5 GiB (profiles/r06/window_bench_payload_cols*.jsonl).  `slot` bounds a
// row (one ring slot), `slack` is the bytes after the last row.
constexpr uint64_t kStreamChunkMax = 256ull << 20;
inline void stream_geometry(uint64_t L, uint64_t count, uint64_t budget, uint64_t min_win, uint64_t slot,
                            uint64_t slack, uint64_t* col, uint64_t* win) {
    const uint64_t half = std::min<uint64_t>(budget / 2, kStreamChunkMax);
    const uint64_t lpad = std::min<uint64_t>((L + 63) / 64 * 64, slot);
    uint64_t w = std::min<uint64_t>(count, min_win);
    const uint64_t per = half > slack && w ? (half - slack) / w : 0;
    const uint64_t wid = per > 256 ? per - 256 : 64;
    uint64_t C = std::max<uint64_t>(64, std::min<uint64_t>(wid >= 4096 ? wid / 4096 * 4096 : wid / 64 * 64, lpad));
    if (C == lpad && w < count && half > slack)
        w = std::min<uint64_t>(count, std::max<uint64_t>(w, (half - slack) / (C + 256) / 64 * 64));
    *col = C;
    *win = w;
}

}  // namespace tvi
