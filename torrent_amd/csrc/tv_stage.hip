// tv_stage.hip -- staging from host memory (tv_stage, tv_stage_many), reading back (tv_read) and the synthetic
// device fill (tv_fill_synthetic).
#include <cstring>

#include "tv_ctx.h"

using namespace tvi;

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
    for (uint64_t k = 0; k < n; k++) {
        if (!lens[k]) continue;
        rc = stage_locked(c, linear_offsets[k], srcs[k], lens[k]);
        if (rc) return rc;
    }
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
        // every window from the open one (or the next unhashed one; a new pass: the first) is filled in its buffer
        // and hashed when the next opens, all on the compute stream
        uint64_t w = c->win_done ? 0 : (c->win_cur != UINT64_MAX ? c->win_cur : (c->win_valid + c->win_n - 1) / c->win_n);
        for (const uint64_t nwin = (c->count + c->win_n - 1) / c->win_n; w < nwin; w++) {
            rc = win_enter(c, w);
            if (rc) return rc;
            const uint64_t j0 = w * c->win_n;
            TV_HIP(c, tv_launch_fill(win_base(c, c->win_buf), c->stride, c->first + j0,
                                     (uint32_t)std::min(c->win_n, c->count - j0), c->L, seed, c->stream));
        }
        TV_HIP(c, hipStreamSynchronize(c->stream));
        return TV_OK;
    }
    TV_HIP(c, tv_launch_fill(c->d_payload, c->stride, c->first, (uint32_t)c->count, c->L, seed, c->stream));
    TV_HIP(c, hipStreamSynchronize(c->stream));
    return TV_OK;
}

}  // extern "C"
