// tv_stage.hip -- staging from host memory (tv_stage, tv_stage_many), reading back (tv_read) and the synthetic
// device fill (tv_fill_synthetic).
#include <cstring>
#include <thread>

#include "tv_ctx.h"

using namespace tvi;

namespace {

// A caller buffer of tv_stage_many packed into a ring slot: LINEAR [a, b) (inside the shard) from src, at slot
// offset `packed` (which has a's alignment mod 4: the DMA out of the slot is dword-aligned).
struct PackedPart {
    uint64_t a, b;
    const uint8_t* src;
    uint64_t packed;
};

// Buffers shorter than this are packed into ring slots without asking whether they are page-locked (a
// hipPointerGetAttributes per buffer costs microseconds, more than copying a small buffer); longer ones are
// checked, and DMA'd directly when they are.
constexpr uint64_t kPackMax = 16ull << 20;

// Stage LINEAR [a, b) from `src` (in a ring slot of `lane`), window by window on a windowed layout (as
// stage_locked; windowed layouts stage on lane 0 only).
int stage_ring_run(tv_ctx* c, uint64_t a, uint64_t b, const uint8_t* src, int lane) {
    if (!c->win) return stage_range(c, a, b, src, a, true, lane, /*src_in_ring=*/true);
    for (uint64_t pos = a; pos < b;) {
        const uint64_t w = win_of(c, pos / c->L - c->first);
        int rc = win_enter(c, w);
        if (rc) return rc;
        uint64_t wa, wb;
        clip_to_shard(c, pos, b - pos, &wa, &wb);
        if (wa < wb) {
            rc = stage_range(c, wa, wb, src, a, true, lane, /*src_in_ring=*/true);
            if (rc) return rc;
        }
        pos = win_end_linear(c, w);
    }
    return TV_OK;
}

// Short buffers packed into the ring slots of one staging lane: add() places a buffer at the next offset with its
// linear offset's alignment mod 4 (a full slot is flushed first); flush() copies the slot's buffers in on the lane's
// pool (a task per buffer, long ones in 4 MiB pieces) and queues one DMA per run of linear-contiguous buffers.
struct Packer {
    tv_ctx* c;
    int lane, threads;
    std::vector<PackedPart> parts;
    uint64_t used = 0;

    int add(uint64_t a, uint64_t b, const uint8_t* src) {
        uint64_t at = used + ((a - used) & 3);
        if (at + (b - a) > kRingSlotBytes) {
            const int rc = flush();
            if (rc) return rc;
            at = a & 3;
        }
        parts.push_back({a, b, src, at});
        used = at + (b - a);
        return TV_OK;
    }
    int flush() {
        used = 0;
        if (parts.empty()) return TV_OK;
        SlotLease slot(c, lane);  // lent until every copy out of it is queued
        int rc = slot.take();
        if (rc) return rc;
        uint8_t* base = slot.ptr();
        constexpr uint64_t kPart = 4ull << 20;
        std::vector<std::pair<uint32_t, uint64_t>> tasks;  // (part, offset inside it)
        for (uint32_t q = 0; q < parts.size(); q++)
            for (uint64_t o = 0; o < parts[q].b - parts[q].a; o += kPart) tasks.emplace_back(q, o);
        c->pool[lane].run(threads, tasks.size(), [&](uint64_t t) {
            const PackedPart& pp = parts[tasks[t].first];
            const uint64_t o = tasks[t].second, n = std::min(kPart, pp.b - pp.a - o);
            tv_copy_host(base + pp.packed + o, pp.src + o, n);
        });
        for (size_t q = 0; q < parts.size();) {
            size_t r = q + 1;
            while (r < parts.size() && parts[r].a == parts[r - 1].b &&
                   parts[r].packed == parts[r - 1].packed + (parts[r - 1].b - parts[r - 1].a))
                r++;
            rc = stage_ring_run(c, parts[q].a, parts[r - 1].b, base + parts[q].packed, lane);
            if (rc) return rc;
            q = r;
        }
        parts.clear();
        return slot.release();
    }
};

}  // namespace

extern "C" {


int tv_stage(tv_ctx* c, uint64_t linear_offset, const uint8_t* src, uint64_t len) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (!src && len) return fail(c, TV_ERR_ARG, "src is NULL");
    if (linear_offset + len < linear_offset) return fail(c, TV_ERR_ARG, "offset + len overflows");
    if (c->count == 0 || len == 0) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    DrainGuard drain(c, 0, /*sync_compute=*/false);  // (a window kernel queued here hashes on after the call)
    rc = stage_locked(c, linear_offset, src, len);
    if (rc) return rc;
    TV_HIP(c, hipStreamSynchronize(c->copy_stream));   // report a copy failure as this call's error
    clear_staged(c, linear_offset, len);
    return TV_OK;
}

int tv_stage_many(tv_ctx* c, uint64_t n, const uint64_t* linear_offsets, const uint8_t* const* srcs,
                  const uint64_t* lens) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (n == 0) return TV_OK;
    if (!linear_offsets || !srcs || !lens) return fail(c, TV_ERR_ARG, "NULL argument");
    for (uint64_t k = 0; k < n; k++) {
        if (!srcs[k] && lens[k]) return fail(c, TV_ERR_ARG, "srcs[%llu] is NULL", (unsigned long long)k);
        if (linear_offsets[k] + lens[k] < linear_offsets[k])
            return fail(c, TV_ERR_ARG, "buffer %llu: offset + len overflows", (unsigned long long)k);
    }
    if (c->count == 0) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    DrainGuard drain(c, 0, /*sync_compute=*/false);  // no DMA reads a caller buffer after the call
    // Short pageable buffers (a torrent's small files, Storage.get results) are packed into ring slots, many per slot
    // and copied by the pool, one DMA per run of adjacent bytes: one slot round trip per buffer made 10,000 small
    // buffers a 6 GB/s path.  Long or page-locked ones go as tv_stage sends them.  Caller order is kept within a lane.
    // When every buffer is short and they fill at least two slots (and the payload is the whole shard: windows must
    // ascend), the second half (by bytes, in caller order) goes to staging lane 1 on a helper thread, as
    // tv_stage_files deals its segments, each lane with half of the context's threads.
    uint64_t small_bytes = 0;
    bool all_small = true;
    for (uint64_t k = 0; k < n; k++) {
        uint64_t a, b;
        clip_to_whole_shard(c, linear_offsets[k], lens[k], &a, &b);
        if (a >= b) continue;
        if (b - a >= kPackMax) all_small = false;
        small_bytes += b - a;
    }
    const bool two = all_small && c->file_concurrent && c->file_threads >= 2 && !c->win && !c->slots &&
                     small_bytes >= 2 * (uint64_t)kRingSlotBytes;
    uint64_t mid = n;
    if (two) {
        uint64_t acc = 0;
        for (mid = 0; mid < n && acc < small_bytes / 2; mid++) {
            uint64_t a, b;
            clip_to_whole_shard(c, linear_offsets[mid], lens[mid], &a, &b);
            if (a < b) acc += b - a;
        }
    }
    const int threads = two ? std::max(1, c->file_threads / 2) : c->file_threads;
    // the buffers [k0, k1) on `lane`
    auto run = [&](uint64_t k0, uint64_t k1, int lane) -> int {
        Packer pk{c, lane, threads};
        for (uint64_t k = k0; k < k1; k++) {
            if (!lens[k]) continue;
            uint64_t a, b;
            clip_to_whole_shard(c, linear_offsets[k], lens[k], &a, &b);
            if (a >= b) continue;
            int rc2;
            if (b - a >= kPackMax) {   // (stage_locked DMAs a page-locked one directly, bounces a pageable one)
                rc2 = pk.flush();
                if (!rc2) rc2 = stage_locked(c, linear_offsets[k], srcs[k], lens[k]);
            } else {
                rc2 = pk.add(a, b, srcs[k] + (a - linear_offsets[k]));
            }
            if (rc2) return rc2;
        }
        return pk.flush();
    };
    int helper_rc = TV_OK;
    std::thread helper;
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{helper};  // every exit joins the helper before the ctx lock is released
    if (two && mid < n) {
        helper = std::thread([&]() {
            pin_thread(numa_cpus(c));  // next to its ring and the GPU
            if (hipSetDevice(c->device) != hipSuccess) {
                helper_rc = fail(c, TV_ERR_HIP, "tv_stage_many: hipSetDevice(%d) failed", c->device);
                return;
            }
            DrainGuard drain1(c, 1, /*sync_compute=*/false);
            helper_rc = run(mid, n, 1);
            if (!helper_rc && hipStreamSynchronize(c->copy_stream2) != hipSuccess)
                helper_rc = fail(c, TV_ERR_HIP, "tv_stage_many: a copy on staging lane 1 failed");
        });
    }
    rc = run(0, mid, 0);
    if (helper.joinable()) helper.join();
    if (rc) return rc;
    if (helper_rc) return helper_rc;
    TV_HIP(c, hipStreamSynchronize(c->copy_stream));
    for (uint64_t k = 0; k < n; k++)
        if (lens[k]) clear_staged(c, linear_offsets[k], lens[k]);
    return TV_OK;
}

int tv_read(tv_ctx* c, uint64_t linear_offset, uint8_t* dst, uint64_t len) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (!dst && len) return fail(c, TV_ERR_ARG, "dst is NULL");
    if (linear_offset + len < linear_offset) return fail(c, TV_ERR_ARG, "offset + len overflows");
    if (c->count == 0 || len == 0) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    uint64_t pos, b;
    clip_to_whole_shard(c, linear_offset, len, &pos, &b);
    if (c->win && pos < b) {  // a windowed layout holds the open window's bytes only
        uint64_t wa, wb;
        clip_to_shard(c, pos, b - pos, &wa, &wb);
        if (wa != pos || wb != b)
            return fail(c, TV_ERR_STATE, "windowed layout: tv_read reads only the open window's pieces");
    }
    DrainGuard drain(c);  // no D2H copy into dst outlives the call, also on error paths
    while (pos < b) {
        const uint64_t i = pos / c->L, within = pos % c->L;
        const uint64_t plen = piece_len(c, i);
        if (within >= plen) { pos = (i + 1) * c->L; continue; }
        const uint8_t* src = nullptr;
        rc = piece_src(c, i, &src);
        if (rc) return rc;
        src += within;
        uint8_t* out = dst + (pos - linear_offset);
        if (within == 0 && plen == c->L && b - pos >= c->L) {
            uint64_t k = (b - pos) / c->L;
            const uint64_t last_full = (c->total % c->L) ? c->P - 1 : c->P;
            k = std::min<uint64_t>(k, last_full > i ? last_full - i : 1);
            if (c->slots) k = 1;
            TV_HIP(c, hipMemcpy2DAsync(out, c->L, src, c->stride, c->L, k, hipMemcpyDeviceToHost, c->copy_stream));
            pos += k * c->L;
        } else {
            const uint64_t n = std::min(b - pos, plen - within);
            TV_HIP(c, hipMemcpyAsync(out, src, n, hipMemcpyDeviceToHost, c->copy_stream));
            pos += n;
        }
    }
    TV_HIP(c, hipStreamSynchronize(c->copy_stream));
    return TV_OK;
}

int tv_fill_synthetic(tv_ctx* c, uint64_t seed) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (!c->count) return TV_OK;
    if (c->slots) return fail(c, TV_ERR_STATE, "tv_fill_synthetic: a slot pool (TV_OPT_LIST_SLOTS) holds no shard");
    TV_HIP(c, hipSetDevice(c->device));
    if (c->win) {
        // every window from the open one (or the next unhashed one; a new pass: the first) is filled in its buffer on
        // staging lane 0 (after the hash that last read the buffer, as a copy would be) and hashed when the next opens
        uint64_t w = c->win_done ? 0 : (c->win_cur != UINT64_MAX ? c->win_cur : (c->win_valid + c->win_n - 1) / c->win_n);
        for (const uint64_t nwin = (c->count + c->win_n - 1) / c->win_n; w < nwin; w++) {
            rc = win_enter(c, w);
            if (rc) return rc;
            const uint64_t j0 = w * c->win_n;
            TV_HIP(c, tv_launch_fill(win_base(c, c->win_buf), c->stride, c->first + j0,
                                     (uint32_t)std::min(c->win_n, c->count - j0), c->L, seed, c->copy_stream));
        }
        TV_HIP(c, hipStreamSynchronize(c->copy_stream));
        TV_HIP(c, hipStreamSynchronize(c->stream));
        return TV_OK;
    }
    TV_HIP(c, tv_launch_fill(c->d_payload, c->stride, c->first, (uint32_t)c->count, c->L, seed, c->stream));
    TV_HIP(c, hipStreamSynchronize(c->stream));
    return TV_OK;
}

}  // extern "C"
