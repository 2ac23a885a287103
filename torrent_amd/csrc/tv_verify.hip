// tv_verify.hip -- the verify and hash calls (tv_verify, tv_verify_list, tv_hash): one launch over the resident
// shard, a list of resident / slotted pieces, or the compare that ends a windowed pass.
#include <cstring>

#include "tv_ctx.h"

using namespace tvi;

extern "C" {

int tv_verify(tv_ctx* c, const uint8_t* avail_bits, uint8_t* bitfield_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, true, true);
    if (rc) return rc;
    if (!bitfield_out && c->count) return fail(c, TV_ERR_ARG, "bitfield_out is NULL");
    if (!c->count) return TV_OK;
    if (c->slots) return fail(c, TV_ERR_STATE, "tv_verify: a slot pool (TV_OPT_LIST_SLOTS) verifies with tv_verify_list");
    TV_HIP(c, hipSetDevice(c->device));
    const uint64_t* av = nullptr;
    if (c->win) {
        // windowed: end the pass (its windows hashed into d_hash as they filled), then compare the whole shard
        rc = win_finalize(c);
        if (!rc) rc = launch_avail(c, avail_bits, &av);
        if (rc) return rc;
        TV_HIP(c, tv_launch_compare(c->d_hash, c->d_digests, (uint32_t)c->count, (uint32_t)c->count, av, c->d_out,
                                    c->stream));
        rc = read_bits(c, bitfield_out);
        if (rc) return rc;
        c->last_launches = (int)c->win_launched;
        return finish_timing(c);
    }
    TV_HIP(c, hipEventRecord(c->ev_call0, c->stream));
    rc = launch_avail(c, avail_bits, &av);
    if (rc) return rc;
    const int kernel = choose_kernel(c);
    TvPieces p = resident_launch(c);
    p.avail64 = av;
    // fail closed: a piece the launch does not write reads as 0, never as a stale 1
    TV_HIP(c, hipMemsetAsync(c->d_out, 0, c->bit_words * 8, c->stream));
    TV_HIP(c, hipEventRecord(c->ev_k0, c->stream));
    rc = launch_resident(c, p, kernel, false);
    if (rc) return rc;
    TV_HIP(c, hipEventRecord(c->ev_k1, c->stream));
    rc = read_bits(c, bitfield_out);
    if (rc) return rc;
    c->last_kernel = kernel;
    c->last_launches = 1;
    return finish_timing(c);
}

int tv_verify_list(tv_ctx* c, const uint64_t* pieces, uint64_t n, uint8_t* ok_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, true, true);
    if (rc) return rc;
    if (n == 0) return TV_OK;
    if (!pieces || !ok_out) return fail(c, TV_ERR_ARG, "NULL argument");
    if (n >= 0xFFFFFFFFull) return fail(c, TV_ERR_ARG, "list too long");
    if (c->win)
        return fail(c, TV_ERR_STATE, "tv_verify_list needs the shard resident or a slot pool (TV_OPT_LIST_SLOTS); "
                                     "this layout is windowed (the shard exceeds the device budget)");
    std::vector<uint32_t> local(n);
    for (uint64_t k = 0; k < n; k++) {
        if (pieces[k] < c->first || pieces[k] >= c->first + c->count)
            return fail(c, TV_ERR_ARG, "piece %llu is not in this context's shard [%llu, %llu)",
                        (unsigned long long)pieces[k], (unsigned long long)c->first,
                        (unsigned long long)(c->first + c->count));
        local[k] = (uint32_t)(pieces[k] - c->first);
    }
    // The entries launched: every listed piece, or, in a slot pool, the listed pieces that hold a slot (the others
    // were never staged: 0).  A short last piece (piece.ts:16-19) listed together with full pieces goes into waves
    // of its own: the launch list is [full pieces..., padding to a multiple of 64, last-piece entries...], so no
    // wave mixes the short piece's padding blocks with the others' raw blocks (the slow path).
    std::vector<uint64_t> sel;
    sel.reserve(n);
    for (uint64_t k = 0; k < n; k++) {
        if (!c->slots || c->slot_of.count(local[k])) sel.push_back(k);
        else ok_out[k] = 0;
    }
    const uint64_t lastj = c->first + c->count - 1 == c->P - 1 ? c->count - 1 : UINT64_MAX;
    uint64_t nlast = 0;
    if (lastj != UINT64_MAX && piece_len(c, c->P - 1) != c->L)
        for (uint64_t k : sel) nlast += local[k] == lastj;
    std::vector<uint32_t> launch;  // shard-relative pieces in launch order (then, for a slot pool, their slots)
    std::vector<int64_t> origin;   // launch position -> index in `pieces` (-1 = padding)
    launch.reserve(sel.size() + 64);
    origin.reserve(sel.size() + 64);
    const bool separate = nlast && nlast < sel.size();
    for (int part = 0; part < (separate ? 2 : 1); part++) {
        for (uint64_t k : sel)
            if (!separate || (local[k] == lastj) == (part == 1)) {
                launch.push_back(local[k]);
                origin.push_back((int64_t)k);
            }
        if (separate && part == 0)
            while (launch.size() % 64) {
                launch.push_back(launch[0]);
                origin.push_back(-1);
            }
    }
    const uint64_t m = launch.size();
    if (c->slots)  // the rows: each entry's slot (the kernels read piece launch[j]'s bytes from slot rows[j])
        for (uint64_t j = 0; j < m; j++) launch.push_back(c->slot_of.find(launch[j])->second);
    std::vector<uint8_t> ok_launch(m);
    TV_HIP(c, hipSetDevice(c->device));
    int kernel = 0;
    if (m) {
        DrainGuard drain(c);  // after the host vectors: their H2D / D2H copies end before they go
        if (c->list_cap < m) {
            free_list(c);
            const uint64_t cap = std::max<uint64_t>(m, 1024);
            TV_HIP(c, hipMalloc((void**)&c->d_list, 2 * cap * 4));  // indices, then (slot pool) rows
            TV_HIP(c, hipMalloc((void**)&c->d_list_out, cap));
            c->list_cap = cap;
            c->n_device_allocs += 2;
        }
        TV_HIP(c, hipEventRecord(c->ev_call0, c->stream));
        TV_HIP(c, hipMemcpyAsync(c->d_list, launch.data(), launch.size() * 4, hipMemcpyHostToDevice, c->stream));
        TvPieces p = resident_launch(c);
        p.n = (uint32_t)m;
        p.n_main = (uint32_t)m;
        p.idx = c->d_list;
        p.rows = c->slots ? c->d_list + m : nullptr;
        p.clock = nullptr;
        p.out_bytes = c->d_list_out;
        TV_HIP(c, hipEventRecord(c->ev_k0, c->stream));
        // twin (two lanes per piece) while its 2-wave workgroups fit two per CU, then split (rounds + helper pair,
        // ~30 % shorter serial stream per block than lane) while one pair per CU suffices, like choose_kernel;
        // the lane list kernel for longer lists
        kernel = (c->kernel_opt == TV_KERNEL_LANE || c->kernel_opt == TV_KERNEL_SPLIT ||
                  c->kernel_opt == TV_KERNEL_TWIN)
                     ? c->kernel_opt
                     : (m <= 64 * (uint64_t)c->cus ? TV_KERNEL_TWIN : (m <= 256 * 64 ? TV_KERNEL_SPLIT : TV_KERNEL_LANE));
        // Companions (as resident launches) only for a list that gives every CU a workgroup: a shorter one would
        // fill 2 x CUs workgroups with copies re-hashing the same few pieces (a 1-piece flush: 512 copies) for a
        // ~4 % shorter flush (r03 latency: tools/latency_probe.py)
        const uint64_t list_wgs = (m + 31) / 32;
        if (kernel == TV_KERNEL_TWIN && (c->twin_fill == 2 || ((c->twin_fill == 1 || c->twin_fill == 3) &&
                                                                list_wgs >= (uint64_t)c->cus && companions_on(c)))) {
            p.fill_to = 2u * (uint32_t)c->cus;
            p.fill_all = c->fill_all ? 1u : 0u;
        }
        TV_HIP(c, tv_launch_verify_list(p, kernel, c->stream, &c->last_workgroups));
        TV_HIP(c, hipEventRecord(c->ev_k1, c->stream));
        TV_HIP(c, hipMemcpyAsync(ok_launch.data(), c->d_list_out, m, hipMemcpyDeviceToHost, c->stream));
        TV_HIP(c, hipEventRecord(c->ev_call1, c->stream));
        TV_HIP(c, hipEventSynchronize(c->ev_call1));
    }
    for (uint64_t i = 0; i < m; i++)
        if (origin[i] >= 0) ok_out[origin[i]] = ok_launch[i];
    if (c->any_file_bad)  // pieces file staging could not read (recover_segment) are 0 here too
        for (uint64_t k = 0; k < n; k++)
            if (get_bit(c->file_bad.data(), local[k])) ok_out[k] = 0;
    if (c->slots)  // a listed piece's slot is free again (a failed piece is staged anew when it is re-downloaded)
        for (uint64_t k = 0; k < n; k++) {
            auto it = c->slot_of.find(local[k]);
            if (it == c->slot_of.end()) continue;
            c->slot_free.push_back(it->second);
            c->slot_of.erase(it);
        }
    c->last_kernel = kernel;
    c->last_launches = m ? 1 : 0;
    if (!m) {
        c->kernel_ms = c->total_ms = 0.f;
        return TV_OK;
    }
    return finish_timing(c);
}

int tv_hash(tv_ctx* c, uint8_t* digests_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (!digests_out && c->count) return fail(c, TV_ERR_ARG, "digests_out is NULL");
    if (!c->count) return TV_OK;
    if (c->slots) return fail(c, TV_ERR_STATE, "tv_hash: a slot pool (TV_OPT_LIST_SLOTS) holds no shard");
    TV_HIP(c, hipSetDevice(c->device));
    int kernel = 0;
    if (c->win) {
        rc = win_finalize(c);  // windowed: the windows were hashed into d_hash as they filled
        if (rc) return rc;
        kernel = c->last_kernel;
    } else {
        TV_HIP(c, hipEventRecord(c->ev_call0, c->stream));
        kernel = choose_kernel(c);
        TvPieces p = resident_launch(c);
        p.avail64 = nullptr;
        TV_HIP(c, hipEventRecord(c->ev_k0, c->stream));
        rc = launch_resident(c, p, kernel, true);
        if (rc) return rc;
        TV_HIP(c, hipEventRecord(c->ev_k1, c->stream));
    }
    std::vector<uint32_t> soa(5 * c->count);
    DrainGuard drain(c);  // declared after soa: drains before soa is freed, also on error paths
    TV_HIP(c, hipMemcpyAsync(soa.data(), c->d_hash, soa.size() * 4, hipMemcpyDeviceToHost, c->stream));
    TV_HIP(c, hipEventRecord(c->ev_call1, c->stream));
    TV_HIP(c, hipEventSynchronize(c->ev_call1));
    for (uint64_t j = 0; j < c->count; j++)
        for (int k = 0; k < 5; k++) {
            const uint32_t v = soa[(uint64_t)k * c->count + j];
            uint8_t* d = digests_out + 20 * j + 4 * k;
            d[0] = (uint8_t)(v >> 24); d[1] = (uint8_t)(v >> 16); d[2] = (uint8_t)(v >> 8); d[3] = (uint8_t)v;
        }
    c->last_kernel = kernel;
    c->last_launches = c->win ? (int)c->win_launched : 1;
    return finish_timing(c);
}

}  // extern "C"
