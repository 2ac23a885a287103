// tv_context.hip -- the context's lifecycle and settings: tv_create / tv_destroy, options, tv_set_layout (the
// payload: the whole shard, windows, or a slot pool), tv_set_digests, pinned-host helpers, timing and counters.
#include <sched.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "tv_ctx.h"

using namespace tvi;

#ifndef TV_SOURCE_ID
#define TV_SOURCE_ID "unknown"
#endif
// The build's source id (torrent_amd/_build.py source_id), findable in the binary: _native.build_id() reads it, and
// measurements tied to a build (profiles/traffic_*.json) carry it.
extern "C" __attribute__((used, visibility("hidden"))) const char tv_build_id_marker[] = "TV_BUILD_ID=" TV_SOURCE_ID;

extern "C" {


int tv_abi_version(void) { return TV_ABI_VERSION; }

int tv_device_count(int* count) {
    if (!count) return fail(nullptr, TV_ERR_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) n = 0;
    else if (e != hipSuccess) return fail(nullptr, TV_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    *count = n;
    return TV_OK;
}

int tv_cpu_share(uint32_t* cores) {
    if (!cores) return fail(nullptr, TV_ERR_ARG, "cores is NULL");
    cpu_set_t set;
    const int aff = sched_getaffinity(0, sizeof set, &set) == 0 ? std::max(1, CPU_COUNT(&set)) : 1;
    double quota = 0;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long per = 0;
        if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per) quota = atof(q) / (double)per;
        fclose(f);
    } else if (FILE* f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
        long long q = 0, per = 0;
        if (fscanf(f1, "%lld", &q) == 1 && q > 0) {
            if (FILE* f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
                if (fscanf(f2, "%lld", &per) == 1 && per > 0) quota = (double)q / (double)per;
                fclose(f2);
            }
        }
        fclose(f1);
    }
    int n = aff;
    const char* omp = getenv("OMP_NUM_THREADS");
    if (quota > 0) n = std::max(1, std::min(aff, (int)quota));
    else if (omp && *omp && strspn(omp, "0123456789") == strlen(omp) && atoi(omp) > 0) n = std::min(aff, atoi(omp));
    *cores = (uint32_t)n;
    return TV_OK;
}

int tv_create(tv_ctx** out, int device) {
    if (!out) return fail(nullptr, TV_ERR_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    int rc = tv_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n) return fail(nullptr, TV_ERR_ARG, "device %d out of range (%d devices)", device, n);
    tv_ctx* c = new tv_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->win_hs[0], hipStreamNonBlocking);  // (see tv_ctx.h win_hs)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy_stream2, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_call0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_k0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_k1);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_call1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_avail, hipEventDisableTiming);
    for (int k = 0; k < 2; k++) {
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->col_ev[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done_ev[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->win_cp[k], hipEventDisableTiming);
    }
    for (int k = 0; k < tvi::kWinBufsMax; k++)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->win_ev[k], hipEventDisableTiming);
    for (int k = 0; k < tvi::kWinHashStreams - 1; k++)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->win_hs_ev[k], hipEventDisableTiming);
    if (e != hipSuccess) {
        fail(nullptr, TV_ERR_HIP, "tv_create: %s", hipGetErrorString(e));
        tv_destroy(c);
        return TV_ERR_HIP;
    }
    // the GPU's NUMA node: the library's threads and pinned ring go there (TV_OPT_NUMA_BIND, default on); the
    // process's CPUs, taken here on the creating thread before any library thread is pinned, are where the
    // workers go back to when the binding is turned off
    c->proc_cpus_ok = sched_getaffinity(0, sizeof c->proc_cpus, &c->proc_cpus) == 0;
    c->numa_node = gpu_numa_node(device);
    c->kfd_gpu_id = kfd_gpu_id(device);   // (this process's own KFD entry is probed lazily: kfd_check_id)
    c->create_pid = (long)getpid();
    c->numa_cpus_ok = node_cpus(c->numa_node, &c->numa_cpus);
    apply_numa(c);
    *out = c;
    return TV_OK;
}

void tv_destroy(tv_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    if (c->copy_stream2) (void)hipStreamSynchronize(c->copy_stream2);
    if (c->pack_stream) (void)hipStreamSynchronize(c->pack_stream);
    (void)win_sync_streams(c);
    free_device(c);
    for (int s = 0; s < kRingSlots; s++) {
        if (c->ring[s]) (void)hipHostFree(c->ring[s]);
        if (c->ring_ev[s]) (void)hipEventDestroy(c->ring_ev[s]);
        if (c->ring2[s]) (void)hipHostFree(c->ring2[s]);
        if (c->ring2_ev[s]) (void)hipEventDestroy(c->ring2_ev[s]);
    }
    if (c->h_bits) (void)hipHostFree(c->h_bits);
    if (c->d_clock) (void)hipFree(c->d_clock);
    for (auto& lane : c->bounce)
        for (auto& b : lane) {
            if (b.ev) (void)hipEventSynchronize(b.ev);
            if (b.ptr) (void)hipHostFree(b.ptr);
            if (b.ev) (void)hipEventDestroy(b.ev);
        }
    for (hipEvent_t ev : {c->ev_call0, c->ev_k0, c->ev_k1, c->ev_call1, c->ev_avail, c->col_ev[0], c->col_ev[1],
                          c->done_ev[0], c->done_ev[1], c->ev_fork, c->ev_join, c->win_cp[0], c->win_cp[1]})
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : c->win_ev)
        if (ev) (void)hipEventDestroy(ev);
    for (int k = 0; k < tvi::kWinHashStreams - 1; k++) {
        if (c->win_hs_ev[k]) (void)hipEventDestroy(c->win_hs_ev[k]);
        if (c->win_hs[k]) (void)hipStreamDestroy(c->win_hs[k]);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->copy_stream2) (void)hipStreamDestroy(c->copy_stream2);
    if (c->pack_stream) (void)hipStreamDestroy(c->pack_stream);
    delete c;
}

int tv_last_error(const tv_ctx* c, char* buf, size_t n) {
    std::string s;
    if (c) {  // a tv_stage_files helper thread may be writing it (fail() takes err_mu)
        std::lock_guard<std::mutex> g(const_cast<tv_ctx*>(c)->err_mu);
        s = c->err;
    } else {
        s = g_thread_error;
    }
    if (buf && n) {
        size_t k = std::min(n - 1, s.size());
        memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int)s.size();
}

int tv_set_option(tv_ctx* c, int key, int64_t value) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    switch (key) {
        case TV_OPT_KERNEL:
            if (value < 0 || value > 4 || value == 3)   // (3 was MIX, removed)
                return fail(c, TV_ERR_ARG, "TV_OPT_KERNEL must be 0 (auto), 1 (lane), 2 (split) or 4 (twin)");
            c->kernel_opt = (int)value;
            return TV_OK;
        case TV_OPT_STRIDE_PAD:
            if (value < 64 || value % 64) return fail(c, TV_ERR_ARG, "TV_OPT_STRIDE_PAD must be a multiple of 64, >= 64");
            if (c->has_layout) return fail(c, TV_ERR_STATE, "TV_OPT_STRIDE_PAD must be set before tv_set_layout");
            c->pad = (uint64_t)value;
            return TV_OK;
        case TV_OPT_STREAM_CHUNK:
            if (value < 0 || value % 64) return fail(c, TV_ERR_ARG, "TV_OPT_STREAM_CHUNK must be a multiple of 64");
            c->stream_chunk = (uint64_t)value;
            return TV_OK;
        case TV_OPT_SPLIT_PAIRS:
            if (value < 0 || value > 5) return fail(c, TV_ERR_ARG, "TV_OPT_SPLIT_PAIRS must be 0 .. 5");
            c->split_pairs = (int)value;
            return TV_OK;
        case TV_OPT_FILE_DIRECT:
            if (value < 0 || value > 1) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_DIRECT must be 0 or 1");
            c->file_direct = value != 0;
            return TV_OK;
        case TV_OPT_FILE_CHUNK:
            if (value < (64 << 10)) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_CHUNK must be >= 65536");
            c->file_chunk = (uint64_t)value;
            return TV_OK;
        case TV_OPT_FILE_DIRECT_MIN:
            if (value < 0) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_DIRECT_MIN must be >= 0");
            c->file_direct_min = (uint64_t)value;
            return TV_OK;
        case TV_OPT_FILE_THREADS:
            if (value < 1 || value > 256) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_THREADS must be 1 .. 256");
            c->file_threads = (int)value;
            return TV_OK;
        case TV_OPT_FILE_CONCURRENT:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_CONCURRENT must be 0 or 1");
            c->file_concurrent = value != 0;
            return TV_OK;
        case TV_OPT_FILE_ODIRECT:
            if (value < 0 || value > 2) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_ODIRECT must be 0, 1 or 2");
            c->file_odirect = (int)value;
            return TV_OK;
        case TV_OPT_RESIDENT:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_RESIDENT must be 0 or 1");
            c->resident = value != 0;  // takes effect at the next tv_set_layout
            return TV_OK;
        case TV_OPT_DEBUG_REBOUNCE:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_DEBUG_REBOUNCE must be 0 or 1");
            c->debug_rebounce = value != 0;
            return TV_OK;
        case TV_OPT_TWIN_PACK:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_TWIN_PACK must be 0 or 1");
            c->twin_pack = value != 0;
            return TV_OK;
        case TV_OPT_TWIN_FILL:
            if (value < 0 || value > 3) return fail(c, TV_ERR_ARG, "TV_OPT_TWIN_FILL must be 0, 1, 2 or 3");
            c->twin_fill = (int)value;
            return TV_OK;
        case TV_OPT_TWIN_FILL_READS:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_TWIN_FILL_READS must be 0 or 1");
            c->fill_all = value != 0;
            return TV_OK;
        case TV_OPT_NUMA_BIND:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_NUMA_BIND must be 0 or 1");
            c->numa_bind = value != 0;
            apply_numa(c);
            return TV_OK;
        case TV_OPT_RESIDENT_BUDGET:
            if (value < 0) return fail(c, TV_ERR_ARG, "TV_OPT_RESIDENT_BUDGET must be >= 0 (0 = automatic)");
            c->budget_opt = (uint64_t)value;  // takes effect at the next tv_set_layout
            return TV_OK;
        case TV_OPT_LIST_SLOTS:
            if (value < 0 || value >= 0xFFFFFFFFll) return fail(c, TV_ERR_ARG, "TV_OPT_LIST_SLOTS must be >= 0 (0 = off)");
            c->list_slots_opt = (uint64_t)value;  // takes effect at the next tv_set_layout
            return TV_OK;
        case TV_OPT_OPEN_RW:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_OPEN_RW must be 0 or 1");
            c->open_rw = value != 0;
            return TV_OK;
        case TV_OPT_LANE_PAIRS:
            if (value < 0 || value > 2) return fail(c, TV_ERR_ARG, "TV_OPT_LANE_PAIRS must be 0 (auto), 1 (on) or 2 (off)");
            c->lane_pairs = (int)value;
            return TV_OK;
        case TV_OPT_CLOCK_PROBE:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_CLOCK_PROBE must be 0 or 1");
            if (value && !c->d_clock) {
                TV_HIP(c, hipSetDevice(c->device));
                TV_HIP(c, hipMalloc((void**)&c->d_clock, kClockWords * sizeof(uint64_t)));
                TV_HIP(c, hipMemset(c->d_clock, 0, kClockWords * sizeof(uint64_t)));
            }
            c->clock_probe = value != 0;
            return TV_OK;
        case TV_OPT_FILE_CLOCK_RESET:
            for (auto& v : c->file_ns) v.store(0);
            return TV_OK;
        case TV_OPT_FILE_BOUNCE:
            if (value < 0 || value > 16) return fail(c, TV_ERR_ARG, "TV_OPT_FILE_BOUNCE must be 0 (off) .. 16 readers");
            c->file_bounce = (int)value;
            return TV_OK;
        case TV_OPT_STREAM_COLD_WINDOW:
            if (value < 0 || value % 64 || value > (1ll << 32))
                return fail(c, TV_ERR_ARG, "TV_OPT_STREAM_COLD_WINDOW must be 0 (default) or a multiple of 64 pieces");
            c->stream_cold_window = (uint64_t)value;
            return TV_OK;
        case TV_OPT_STREAM_COLD_READERS:
            if (value < 0 || value > 256) return fail(c, TV_ERR_ARG, "TV_OPT_STREAM_COLD_READERS must be 0 .. 256");
            c->stream_cold_readers = (int)value;
            return TV_OK;
        case TV_OPT_STREAM_COLD_REQ:
            if (value < 0 || (value > 0 && value < 4096)) return fail(c, TV_ERR_ARG, "TV_OPT_STREAM_COLD_REQ must be 0 or >= 4096");
            c->stream_cold_req = (uint64_t)value;
            return TV_OK;
        case TV_OPT_WIN_BUFS:
            if (value < 0 || value > kWinBufsMax)
                return fail(c, TV_ERR_ARG, "TV_OPT_WIN_BUFS must be 0 (default) .. %d", kWinBufsMax);
            c->win_bufs_opt = (int)value;   // takes effect at the next tv_set_layout
            return TV_OK;
        case TV_OPT_WIN_STREAMS:
            if (value < 0 || value > kWinHashStreams)
                return fail(c, TV_ERR_ARG, "TV_OPT_WIN_STREAMS must be 0 (default) .. %d", kWinHashStreams);
            c->win_streams_opt = (int)value;   // takes effect at the next tv_set_layout
            return TV_OK;
        case TV_OPT_STREAM_ROWS:
            if (value != 0 && value != 1) return fail(c, TV_ERR_ARG, "TV_OPT_STREAM_ROWS must be 0 or 1");
            if (c->st.active) return fail(c, TV_ERR_STATE, "TV_OPT_STREAM_ROWS cannot change during a stream");
            c->stream_rows = value != 0;
            return TV_OK;
    }
    return fail(c, TV_ERR_ARG, "unknown option %d", key);
}

int tv_get_option(tv_ctx* c, int key, int64_t* value) {
    if (!c || !value) return fail(c, TV_ERR_ARG, "NULL argument");
    std::lock_guard<std::mutex> g(c->mu);
    switch (key) {
        case TV_OPT_KERNEL: *value = c->kernel_opt; return TV_OK;
        case TV_OPT_STRIDE_PAD: *value = (int64_t)c->pad; return TV_OK;
        case TV_OPT_STREAM_CHUNK: *value = (int64_t)c->stream_chunk; return TV_OK;
        case TV_OPT_SPLIT_PAIRS: *value = c->split_pairs; return TV_OK;
        case TV_OPT_FILE_DIRECT: *value = c->file_direct ? 1 : 0; return TV_OK;
        case TV_OPT_FILE_CHUNK: *value = (int64_t)c->file_chunk; return TV_OK;
        case TV_OPT_FILE_DIRECT_MIN: *value = (int64_t)c->file_direct_min; return TV_OK;
        case TV_OPT_FILE_THREADS: *value = c->file_threads; return TV_OK;
        case TV_OPT_FILE_CONCURRENT: *value = c->file_concurrent ? 1 : 0; return TV_OK;
        case TV_OPT_FILE_ODIRECT: *value = c->file_odirect; return TV_OK;
        case TV_OPT_RESIDENT: *value = c->resident ? 1 : 0; return TV_OK;
        case TV_OPT_DEBUG_REBOUNCE: *value = c->debug_rebounce ? 1 : 0; return TV_OK;
        case TV_OPT_TWIN_PACK: *value = c->twin_pack ? 1 : 0; return TV_OK;
        case TV_OPT_TWIN_FILL: *value = c->twin_fill; return TV_OK;
        case TV_OPT_TWIN_FILL_READS: *value = c->fill_all ? 1 : 0; return TV_OK;
        case TV_OPT_NUMA_BIND: *value = c->numa_bind ? 1 : 0; return TV_OK;
        case TV_OPT_RESIDENT_BUDGET: *value = (int64_t)c->budget_opt; return TV_OK;
        case TV_OPT_LIST_SLOTS: *value = (int64_t)c->list_slots_opt; return TV_OK;
        case TV_OPT_OPEN_RW: *value = c->open_rw ? 1 : 0; return TV_OK;
        case TV_OPT_STREAM_ROWS: *value = c->stream_rows ? 1 : 0; return TV_OK;
        case TV_OPT_CLOCK_PROBE: *value = c->clock_probe ? 1 : 0; return TV_OK;
        case TV_OPT_LANE_PAIRS: *value = c->lane_pairs; return TV_OK;
        case TV_OPT_WIN_BUFS: *value = c->win_bufs_opt; return TV_OK;
        case TV_OPT_FILE_BOUNCE: *value = c->file_bounce; return TV_OK;
        case TV_OPT_STREAM_COLD_WINDOW: *value = (int64_t)c->stream_cold_window; return TV_OK;
        case TV_OPT_STREAM_COLD_READERS: *value = c->stream_cold_readers; return TV_OK;
        case TV_OPT_STREAM_COLD_REQ: *value = (int64_t)c->stream_cold_req; return TV_OK;
        case TV_OPT_WIN_STREAMS: *value = c->win_streams_opt; return TV_OK;
    }
    return fail(c, TV_ERR_ARG, "unknown option %d", key);
}

int tv_set_layout(tv_ctx* c, uint64_t total_length, uint64_t piece_length, uint64_t n_pieces,
                  uint64_t shard_first, uint64_t shard_count) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (piece_length == 0) return fail(c, TV_ERR_ARG, "piece_length must be > 0");
    if (shard_first > n_pieces || shard_count > n_pieces - shard_first)
        return fail(c, TV_ERR_ARG, "shard [%llu, +%llu) outside %llu pieces", (unsigned long long)shard_first,
                    (unsigned long long)shard_count, (unsigned long long)n_pieces);
    // (an empty shard has no bitfield slice, so it may start anywhere: a trailing empty shard of
    // shard_ranges starts at P, which need not be a multiple of 8)
    if (shard_first % 8 && shard_count)
        return fail(c, TV_ERR_ARG, "shard_first must be a multiple of 8 (whole bitfield bytes)");
    if (shard_count >= 0xFFFFFFFFull) return fail(c, TV_ERR_ARG, "shard_count too large");
    if (piece_length > (1ull << 36)) return fail(c, TV_ERR_ARG, "piece_length must be <= 64 GiB");
    // every linear offset i*L (+L) and digest offset 20*i (+20) of the torrent must fit in 64 bits, and so
    // must the resident allocation; otherwise a wrapped offset would index the wrong bytes
    const uint64_t stride = ((piece_length + 63) / 64) * 64 + c->pad;
    if (n_pieces >= UINT64_MAX / 20 || n_pieces >= UINT64_MAX / piece_length - 1 ||
        (shard_count && shard_count > (UINT64_MAX - kSlack) / stride))
        return fail(c, TV_ERR_ARG, "geometry overflows 64-bit offsets (%llu pieces of %llu bytes)",
                    (unsigned long long)n_pieces, (unsigned long long)piece_length);
    TV_HIP(c, hipSetDevice(c->device));
    stream_abort_locked(c);
    TV_HIP(c, hipStreamSynchronize(c->stream));
    TV_HIP(c, hipStreamSynchronize(c->copy_stream));
    TV_HIP(c, hipStreamSynchronize(c->copy_stream2));
    {
        const int rc = win_sync_streams(c);   // (a window hash of the last layout may still read the payload)
        if (rc) return rc;
    }
    c->has_layout = false;
    c->digests_set = false;
    c->total = total_length;
    c->L = piece_length;
    c->P = n_pieces;
    c->first = shard_first;
    c->count = shard_count;
    c->stride = stride;
    c->bit_words = ((shard_count + 255) / 256) * 4;
    c->digest_ok.assign((shard_count + 7) / 8 + 8, 0);
    c->file_bad.assign((shard_count + 7) / 8 + 8, 0);
    c->any_file_bad = false;
    c->unhashed.assign((shard_count + 7) / 8 + 8, 0);
    c->any_unhashed = false;
    c->win = false;
    c->win_n = 0;
    c->win_bufs = 0;
    c->win_nhs = 1;
    c->win_buf_bytes = 0;
    c->win_cur = UINT64_MAX;
    c->win_buf = 1;
    c->win_valid = 0;
    c->win_done = false;
    c->win_timing = false;
    c->win_launched = 0;
    c->win_passes = 0;
    c->slots = 0;
    c->slot_of.clear();
    c->slot_free.clear();
    c->budget = 0;
    // Keep every allocation the new geometry fits (reuse_fits): a run of small layouts (verify_piece,
    // a flush of tv_verify_list) allocates once.  Everything else is released first, so a big payload
    // is never held beside its replacement.
    // A layout without a resident payload (TV_OPT_RESIDENT = 0) releases the old one: the resident calls must
    // see no payload (TV_ERR_STATE), never a smaller buffer left by an earlier layout.  The streamed path's
    // chunk buffers are kept only for a streamed layout they fit (a resident payload must not be allocated
    // beside them), and the list buffers only while they are not far larger than the shard.
    uint64_t need_payload = (shard_count && c->resident) ? shard_count * c->stride + kSlack : 0;
    uint64_t budget = 0;
    if (need_payload && c->list_slots_opt) {
        // a slot pool (incremental verify): K piece slots, whatever the shard's size
        c->slots = std::min<uint64_t>(c->list_slots_opt, shard_count);
        need_payload = c->slots * c->stride + kSlack;
        for (uint64_t q = c->slots; q-- > 0;) c->slot_free.push_back((uint32_t)q);  // slot 0 is taken first
    } else if (need_payload) {
        // The device budget: TV_OPT_RESIDENT_BUDGET, or what HBM has free (plus what this ctx would release) less
        // a margin for the per-piece rows and whatever else shares the GPU
        budget = c->budget_opt;
        if (!budget) {
            size_t fr = 0, tot = 0;
            TV_HIP(c, hipMemGetInfo(&fr, &tot));
            const uint64_t avail = (uint64_t)fr + c->cap_payload + 2 * c->chunk_bytes;
            const uint64_t margin = (4ull << 30) + 64 * shard_count;
            budget = avail > margin ? avail - margin : 0;
        }
    }
    // The payload: the whole shard when it fits the budget, else windows (a torrent of any size on a
    // GPU of any free memory).  A failed allocation is retried at half the budget: only the windows shrink
    // (tv_plan.h allocate_payload; it gives up when the request cannot get smaller).
    if (need_payload && !c->slots) {
        PayloadPlan plan;
        uint64_t failed = 0;
        hipError_t last = hipSuccess;
        const int r = allocate_payload(
            shard_count, c->stride, kSlack, budget,
            [&](const PayloadPlan& p, uint64_t b) -> int {
                // (an allocation larger than the budget is never kept: the budget bounds what the ctx holds)
                if (!reuse_fits(p.bytes, c->cap_payload) || c->cap_payload > b) free_payload(c);
                if (c->d_payload) return 0;
                last = hipMalloc((void**)&c->d_payload, p.bytes);
                if (last == hipSuccess) {
                    c->cap_payload = p.bytes;
                    c->n_payload_allocs++;
                    c->n_device_allocs++;
                    return 0;
                }
                (void)hipGetLastError();
                c->d_payload = nullptr;
                return last == hipErrorOutOfMemory ? 1 : 2;
            },
            &plan, &budget, &failed, c->win_bufs_opt > 0 ? c->win_bufs_opt : kWinBufsDefault);
        if (r)
            return fail(c, r == 1 ? TV_ERR_NOMEM : TV_ERR_HIP, "hipMalloc(%llu) of the payload: %s",
                        (unsigned long long)failed, hipGetErrorString(last));
        need_payload = plan.bytes;
        c->win = plan.win;
        c->win_n = plan.win_n;
        c->win_bufs = plan.bufs;
        c->win_buf_bytes = plan.buf_bytes;
        // hash streams: one per window that may hash while the next one stages (TV_OPT_WIN_STREAMS overrides)
        c->win_nhs = c->win ? std::max(1, std::min(kWinHashStreams, c->win_streams_opt > 0 ? c->win_streams_opt
                                                                                          : plan.bufs - 1))
                            : 1;
        for (int k = 0; k + 1 < c->win_nhs; k++)
            if (!c->win_hs[k]) TV_HIP(c, hipStreamCreateWithFlags(&c->win_hs[k], hipStreamNonBlocking));
    } else {
        if (!need_payload || !reuse_fits(need_payload, c->cap_payload)) free_payload(c);
        if (need_payload && !c->d_payload) {
            TV_HIP(c, hipMalloc((void**)&c->d_payload, need_payload));
            c->cap_payload = need_payload;
            c->n_payload_allocs++;
            c->n_device_allocs++;
        }
    }
    c->budget = budget;
    if (!reuse_fits(shard_count, c->cap_count)) free_per_piece(c);
    if (!reuse_fits(c->bit_words, c->cap_words)) free_words(c);
    if (c->chunk_bytes && (need_payload || !reuse_fits(stream_chunk_need(c), c->chunk_bytes))) free_chunks(c);
    if (c->list_cap > std::max<uint64_t>(1024, 2 * shard_count)) free_list(c);
    if (shard_count && !c->d_digests) {
        TV_HIP(c, hipMalloc((void**)&c->d_digests, 5 * shard_count * sizeof(uint32_t)));
        TV_HIP(c, hipMalloc((void**)&c->d_state, 5 * shard_count * sizeof(uint32_t)));
        TV_HIP(c, hipMalloc((void**)&c->d_hash, 5 * shard_count * sizeof(uint32_t)));
        c->cap_count = shard_count;
        c->n_device_allocs += 3;
    }
    if (shard_count && !c->d_out) {
        TV_HIP(c, hipMalloc((void**)&c->d_avail, c->bit_words * 8));
        TV_HIP(c, hipMalloc((void**)&c->d_base_avail, c->bit_words * 8));
        TV_HIP(c, hipHostMalloc((void**)&c->h_avail, c->bit_words * 8, hipHostMallocDefault));
        TV_HIP(c, hipMalloc((void**)&c->d_out, c->bit_words * 8));
        c->cap_words = c->bit_words;
        c->n_device_allocs += 3;
    }
    if (need_payload) {  // the tail over-read slack past the last piece (of each window buffer, of the slots) reads zeros
        const uint64_t rows = c->win ? c->win_n : (c->slots ? c->slots : shard_count);
        for (int k = 0; k < (c->win ? c->win_bufs : 1); k++)
            TV_HIP(c, hipMemsetAsync(c->d_payload + (uint64_t)k * c->win_buf_bytes + rows * c->stride, 0, kSlack,
                                     c->stream));
        TV_HIP(c, hipStreamSynchronize(c->stream));
    }
    c->has_layout = true;
    return TV_OK;
}

int tv_set_digests(tv_ctx* c, const uint8_t* pieces, uint64_t pieces_len) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->st.active) {
        TV_HIP(c, hipSetDevice(c->device));
        stream_abort_locked(c);
    }
    int rc = require_layout(c, false);
    if (rc) return rc;
    if (!pieces && pieces_len) return fail(c, TV_ERR_ARG, "pieces is NULL");
    c->digests_set = false;  // until the digests AND their base availability are both on the device
    // partition(info.pieces, 20) (metainfo.ts:111, _bytes.ts:92-99): slice i = [20i, 20i+20)
    std::vector<uint32_t> soa(5 * c->count, 0);
    std::fill(c->digest_ok.begin(), c->digest_ok.end(), 0);
    for (uint64_t j = 0; j < c->count; j++) {
        const uint64_t i = c->first + j;
        if (20 * i + 20 > pieces_len) continue;  // short or missing slice: never equal
        const uint8_t* d = pieces + 20 * i;
        for (int k = 0; k < 5; k++)
            soa[(uint64_t)k * c->count + j] = ((uint32_t)d[4 * k] << 24) | ((uint32_t)d[4 * k + 1] << 16) |
                                              ((uint32_t)d[4 * k + 2] << 8) | (uint32_t)d[4 * k + 3];
        set_bit(c->digest_ok.data(), j);
    }
    if (c->count) {
        TV_HIP(c, hipSetDevice(c->device));
        TV_HIP(c, hipMemcpyAsync(c->d_digests, soa.data(), soa.size() * 4, hipMemcpyHostToDevice, c->stream));
        TV_HIP(c, hipStreamSynchronize(c->stream));
    }
    if (c->count) {
        rc = upload_base_avail(c);
        if (rc) return rc;
    }
    c->digests_set = true;
    return TV_OK;
}


int tv_host_alloc(uint64_t bytes, void** out) {
    if (!out) return fail(nullptr, TV_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (bytes == 0) return TV_OK;
    hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
    if (e != hipSuccess)
        return fail(nullptr, e == hipErrorOutOfMemory ? TV_ERR_NOMEM : TV_ERR_HIP, "hipHostMalloc(%llu): %s",
                    (unsigned long long)bytes, hipGetErrorString(e));
    return TV_OK;
}

int tv_host_free(void* ptr) {
    if (!ptr) return TV_OK;
    hipError_t e = hipHostFree(ptr);
    if (e != hipSuccess) return fail(nullptr, TV_ERR_HIP, "hipHostFree: %s", hipGetErrorString(e));
    return TV_OK;
}

int tv_host_register(void* ptr, uint64_t bytes) {
    if (!ptr || !bytes) return fail(nullptr, TV_ERR_ARG, "NULL or empty range");
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
    if (e != hipSuccess) return fail(nullptr, TV_ERR_HIP, "hipHostRegister: %s", hipGetErrorString(e));
    return TV_OK;
}

int tv_host_unregister(void* ptr) {
    if (!ptr) return fail(nullptr, TV_ERR_ARG, "ptr is NULL");
    hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) return fail(nullptr, TV_ERR_HIP, "hipHostUnregister: %s", hipGetErrorString(e));
    return TV_OK;
}

int tv_last_timing(tv_ctx* c, double* kernel_ms, double* total_ms) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (kernel_ms) *kernel_ms = c->kernel_ms;
    if (total_ms) *total_ms = c->total_ms;
    return TV_OK;
}

int tv_get_counter(tv_ctx* c, int key, uint64_t* value) {
    if (!c || !value) return fail(c, TV_ERR_ARG, "NULL argument");
    std::lock_guard<std::mutex> g(c->mu);
    switch (key) {
        case TV_COUNTER_PAYLOAD_ALLOCS: *value = c->n_payload_allocs; return TV_OK;
        case TV_COUNTER_DEVICE_ALLOCS: *value = c->n_device_allocs; return TV_OK;
        case TV_COUNTER_PAYLOAD_BYTES: *value = c->cap_payload; return TV_OK;
        case TV_COUNTER_DEVICE_BYTES:
            *value = c->cap_payload + c->cap_count * 3 * 5 * sizeof(uint32_t) + c->cap_words * 8 * 3 +
                     2 * c->chunk_bytes + c->list_cap * 9;
            return TV_OK;
        case TV_COUNTER_LAST_WORKGROUPS: *value = c->last_workgroups; return TV_OK;
        case TV_COUNTER_NUMA_NODE: *value = c->numa_node < 0 ? UINT64_MAX : (uint64_t)c->numa_node; return TV_OK;
        case TV_COUNTER_RING_NODE: {
            const int node = page_node(c->ring[0]);
            *value = node < 0 ? UINT64_MAX : (uint64_t)node;
            return TV_OK;
        }
        case TV_COUNTER_WINDOW_PIECES: *value = c->win ? c->win_n : 0; return TV_OK;
        case TV_COUNTER_WINDOWS: *value = c->win_launched; return TV_OK;
        case TV_COUNTER_WINDOW_BUFS: *value = c->win ? (uint64_t)c->win_bufs : 0; return TV_OK;
        case TV_COUNTER_WINDOW_STREAMS: *value = c->win ? (uint64_t)c->win_nhs : 0; return TV_OK;
        case TV_COUNTER_BUDGET: *value = c->budget; return TV_OK;
        case TV_COUNTER_SLOTS_USED: *value = c->slot_of.size(); return TV_OK;
        case TV_COUNTER_FILE_CLOCK + TV_FILE_PHASE_OPEN ... TV_COUNTER_FILE_CLOCK + TV_FILE_CLOCK_N - 1:
            *value = c->file_ns[key - TV_COUNTER_FILE_CLOCK].load();
            return TV_OK;
        case TV_COUNTER_COTENANT_VRAM: *value = cotenant_vram(c); return TV_OK;
        case TV_COUNTER_KFD_GPU_ID: *value = kfd_check_id(c); return TV_OK;
        case TV_COUNTER_LAST_CLOCK_KHZ: {
            *value = 0;
            if (!c->d_clock) return TV_OK;
            uint64_t st[4] = {0, 0, 0, 0};
            TV_HIP(c, hipSetDevice(c->device));
            TV_HIP(c, hipStreamSynchronize(c->stream));
            TV_HIP(c, hipMemcpy(st, c->d_clock, sizeof st, hipMemcpyDeviceToHost));
            if (st[3] > st[1] && st[2] > st[0])   // shader cycles / real-time ticks x 100 MHz
                *value = (uint64_t)((double)(st[2] - st[0]) / (double)(st[3] - st[1]) * 100000.0 + 0.5);
            return TV_OK;
        }
    }
    return fail(c, TV_ERR_ARG, "unknown counter %d", key);
}

#if TV_STAMPS
// Diagnostic builds only (not in include/torrent_verify.h): copy the clock buffer (probe + split loop stamps).
int tv_debug_stamps(tv_ctx* c, void* out, uint64_t bytes) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (!out || !c->d_clock) return fail(c, TV_ERR_ARG, "no clock buffer (set TV_OPT_CLOCK_PROBE)");
    if (bytes > kClockWords * sizeof(uint64_t)) bytes = kClockWords * sizeof(uint64_t);
    TV_HIP(c, hipSetDevice(c->device));
    TV_HIP(c, hipStreamSynchronize(c->stream));
    TV_HIP(c, hipMemcpy(out, c->d_clock, bytes, hipMemcpyDeviceToHost));
    return TV_OK;
}
#endif

int tv_last_kernel(tv_ctx* c, int* kernel, int* launches) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (kernel) *kernel = c->last_kernel;
    if (launches) *launches = c->last_launches;
    return TV_OK;
}

int tv_synchronize(tv_ctx* c) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    TV_HIP(c, hipSetDevice(c->device));
    TV_HIP(c, hipStreamSynchronize(c->copy_stream));
    TV_HIP(c, hipStreamSynchronize(c->copy_stream2));
    TV_HIP(c, hipStreamSynchronize(c->stream));
    return TV_OK;
}


}  // extern "C"
