// tv_stream.hip -- the streamed verify engine (tv_stream_*; tv_verify_host runs on it): a bounded pinned ring
// between the caller's bytes and two device chunk buffers, one kernel launch per column / window of pieces.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <memory>

#include "tv_ctx.h"

namespace tvi {

// ---- streamed verify (tv_stream_*; tv_verify_host runs on it too) ------------------------------------
//
// Column `col` carries bytes [col*C, col*C + C) of every shard piece.  Its rows arrive as requests of up to
// one ring slot (64 MiB) each, filled by the caller, and are DMA'd from the slot into device chunk buffer
// col & 1 (row pitch C + 256).  When a column's last request is committed, one kernel launch hashes it on the
// compute stream (chaining values persist in d_state; the last column pads, compares and writes the
// bitfield) while the next column's requests fill the other buffer.  Host memory in flight: the ring.

uint64_t row_bytes(const tv_ctx* c, uint64_t piece, uint64_t offset, uint64_t width) {  // piece.ts:16-19
    const uint64_t plen = piece_len(c, piece);
    return plen > offset ? std::min(width, plen - offset) : 0;
}

// Drop an active stream: give its lent slot back and let the queued copies and kernels drain.
void stream_abort_locked(tv_ctx* c) {
    StreamState& st = c->st;
    if (!st.active) return;
    if (st.outstanding && st.slot >= 0) (void)release_slot(c, st.slot, 0);
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipGetLastError();
    st = StreamState{};
}

// Row mode (TV_OPT_STREAM_ROWS): each request row is a whole piece (one Storage.get per piece), which needs a
// piece to fit one ring slot.
bool stream_rows(const tv_ctx* c) { return c->stream_rows && c->L <= kRingSlotBytes; }

// Row mode's window: whole pieces per chunk buffer, a multiple of 64 (bitfield words of their own), at most
// kRowWindowBytes per buffer (TV_OPT_RESIDENT_BUDGET / 2 if smaller), the shard when it fits.
constexpr uint64_t kRowWindowBytes = 4ull << 30;
uint64_t stream_row_window(const tv_ctx* c) {
    const uint64_t pitch = (c->L + 63) / 64 * 64 + 256;
    uint64_t bytes = kRowWindowBytes;
    if (c->budget_opt) bytes = std::min<uint64_t>(bytes, c->budget_opt / 2);
    const uint64_t w = std::max<uint64_t>(64, bytes / pitch / 64 * 64);
    return std::min<uint64_t>(w, c->count);
}

// Column width: TV_OPT_STREAM_CHUNK, or ~512 MiB columns (64 KiB .. L); a multiple of 64, at most one slot.
uint64_t stream_column(const tv_ctx* c) {
    uint64_t C = c->stream_chunk;
    if (!C) {
        C = 64ull << 10;
        while (C * 2 <= c->L && C * 2 * c->count <= (512ull << 20)) C *= 2;
    }
    C = std::min<uint64_t>((C / 64) * 64, ((c->L + 63) / 64) * 64);
    return std::max<uint64_t>(64, std::min<uint64_t>(C, kRingSlotBytes));
}

// Bytes of each of the two device chunk buffers a stream over the current geometry needs.
uint64_t stream_chunk_need(const tv_ctx* c) {
    if (!c->count) return 0;
    if (stream_rows(c)) return ((c->L + 63) / 64 * 64 + 256) * stream_row_window(c) + kSlack;
    return (stream_column(c) + 256) * c->count + kSlack;
}

// The geometry of a stream under a device budget: tv_plan.h stream_geometry (its rationale there).
void budget_geometry(const tv_ctx* c, uint64_t budget, uint64_t min_win, uint64_t* col, uint64_t* win) {
    stream_geometry(c->L, c->count, budget, min_win, kRingSlotBytes, kSlack, col, win);
}

int stream_begin_locked(tv_ctx* c, const uint8_t* avail_bits, uint64_t col_override = 0, uint64_t win_override = 0,
                        uint64_t req_bytes = 0) {
    StreamState& st = c->st;
    st = StreamState{};
    st.av.assign((c->count + 7) / 8, 0xFF);
    if (avail_bits) memcpy(st.av.data(), avail_bits, st.av.size());
    if (c->count == 0) {  // nothing to hash: the first tv_stream_next reports completion
        st.active = true;
        return TV_OK;
    }
    if (stream_rows(c)) {  // whole pieces per row, windows of wn pieces
        st.C = (c->L + 63) / 64 * 64;
        st.wn = stream_row_window(c);
    } else {               // columns across the whole shard (or across windows of win_override pieces)
        st.C = col_override ? col_override : stream_column(c);
        st.wn = win_override ? std::min(win_override, c->count) : c->count;
    }
    st.row_pitch = st.C + 256;  // (tail over-read slack per row)
    const uint64_t need = st.row_pitch * st.wn + kSlack;
    if (!reuse_fits(need, c->chunk_bytes)) {
        free_chunks(c);
        for (auto& p : c->d_chunk) {
            TV_HIP(c, hipMalloc((void**)&p, need));
            c->n_device_allocs++;
        }
        c->chunk_bytes = need;
    }
    st.ncol = (c->L + st.C - 1) / st.C;
    st.nwin = (c->count + st.wn - 1) / st.wn;
    st.nunits = st.nwin * st.ncol;
    st.rows_per_req = std::max<uint64_t>(1, (req_bytes ? std::min<uint64_t>(req_bytes, kRingSlotBytes) : kRingSlotBytes) / st.C);
    TV_HIP(c, hipEventRecord(c->ev_call0, c->stream));
    TV_HIP(c, hipMemsetAsync(c->d_out, 0, c->bit_words * 8, c->stream));  // fail closed, as tv_verify
    TV_HIP(c, hipEventRecord(c->done_ev[0], c->stream));
    TV_HIP(c, hipEventRecord(c->done_ev[1], c->stream));
    st.active = true;
    return TV_OK;
}

int stream_next_locked(tv_ctx* c, tv_stream_req* req) {
    StreamState& st = c->st;
    if (!st.active) return fail(c, TV_ERR_STATE, "tv_stream_begin has not been called");
    if (st.outstanding)
        return fail(c, TV_ERR_STATE, "request %llu is still outstanding (commit it first)", (unsigned long long)st.req.seq);
    *req = tv_stream_req{};
    if (st.unit >= st.nunits) return TV_OK;  // rows == 0: every byte has been requested
    const int buf = (int)(st.unit & 1);
    const uint64_t j0 = st.unit / st.ncol * st.wn, wcount = std::min(st.wn, c->count - j0);
    // the first copy into chunk buffer `buf` waits for the kernel that last read it
    if (st.row == 0) TV_HIP(c, hipStreamWaitEvent(c->copy_stream, c->done_ev[buf], 0));
    int rc = take_slot(c, &st.slot, 0);
    if (rc) return rc;
    req->piece = c->first + j0 + st.row;
    req->rows = std::min<uint64_t>(st.rows_per_req, wcount - st.row);
    req->offset = st.unit % st.ncol * st.C;
    req->width = std::min<uint64_t>(st.C, c->L - req->offset);
    req->slot = c->ring[st.slot];
    req->seq = ++st.seq;
    st.req = *req;
    st.outstanding = true;
    return TV_OK;
}

// Queue the outstanding request's rows [0, rows_copy) (the others are unreadable and not copied).  Source:
// the request's slot (src == nullptr), or caller memory at src (row q at src + q*pitch), DMA'd directly when
// page-locked and gathered into the slot otherwise.  Completes the column: one kernel launch.
int stream_commit_locked(tv_ctx* c, const tv_stream_req* req, const uint8_t* src, uint64_t pitch, bool pinned,
                         uint64_t rows_copy) {
    StreamState& st = c->st;
    if (!st.active) return fail(c, TV_ERR_STATE, "tv_stream_begin has not been called");
    if (!st.outstanding) return fail(c, TV_ERR_STATE, "no outstanding request (call tv_stream_next)");
    if (!req || req->seq != st.req.seq || req->piece != st.req.piece || req->rows != st.req.rows)
        return fail(c, TV_ERR_ARG, "the request does not match outstanding request %llu", (unsigned long long)st.req.seq);
    const tv_stream_req r = st.req;
    const int buf = (int)(st.unit & 1);
    const uint64_t j0 = st.unit / st.ncol * st.wn, wcount = std::min(st.wn, c->count - j0);
    uint8_t* dst = c->d_chunk[buf] + st.row * st.row_pitch;
    uint8_t* slot = c->ring[st.slot];
    const uint64_t n = std::min(rows_copy, r.rows);
    uint64_t full = n;  // rows [0, full) carry `width` bytes; only the torrent's short last piece has fewer
    if (full && row_bytes(c, r.piece + full - 1, r.offset, r.width) < r.width) full--;
    const uint64_t tail = full < n ? row_bytes(c, r.piece + full, r.offset, r.width) : 0;
    const uint8_t* from = slot;
    uint64_t from_pitch = r.width;
    if (src) {
        if (pinned) {
            from = src;
            from_pitch = pitch;
        } else {
            gather_rows(c->pool[0], slot, src, r.width, pitch, full, c->file_threads);
            if (tail) memcpy(slot + full * r.width, src + full * pitch, tail);
        }
    }
    if (full)
        TV_HIP(c, hipMemcpy2DAsync(dst, st.row_pitch, from, from_pitch, r.width, full, hipMemcpyHostToDevice,
                                   c->copy_stream));
    if (tail)
        TV_HIP(c, hipMemcpyAsync(dst + full * st.row_pitch, from + full * from_pitch, tail, hipMemcpyHostToDevice,
                                 c->copy_stream));
    st.outstanding = false;
    const int s = st.slot;
    st.slot = -1;
    int rc = release_slot(c, s, 0);  // its event follows the copies just queued
    if (rc) return rc;
    st.row += r.rows;
    if (st.row < wcount) return TV_OK;
    // the unit is complete: hash it while the caller fills the next one
    TV_HIP(c, hipEventRecord(c->col_ev[buf], c->copy_stream));
    TV_HIP(c, hipStreamWaitEvent(c->stream, c->col_ev[buf], 0));
    if (!st.k0) {
        TV_HIP(c, hipEventRecord(c->ev_k0, c->stream));
        st.k0 = true;
    }
    const bool last = st.unit % st.ncol + 1 == st.ncol;
    // the window's pieces (the shard's digest / state rows from j0; bitfield words from j0 / 64: a window of a
    // multi-window stream is a multiple of 64 pieces)
    TvPieces p = window_launch(c, j0, wcount, c->d_chunk[buf]);
    p.stride = st.row_pitch;
    p.avail64 = c->d_base_avail + j0 / 64;
    p.out64 = c->d_out + j0 / 64;
    p.data_off = r.offset;
    p.blk_begin = r.offset / 64;
    p.blk_end = last ? UINT64_MAX : (r.offset + st.C) / 64;
    p.finalize = last ? 1 : 0;
    st.kernel = choose_kernel_n(c, wcount, p.n_main < p.n);
    p.lane_pairs = lane_pairs_for(c, p.n);
    TV_HIP(c, tv_launch_verify(p, st.kernel, false, c->stream, c->split_pairs, &c->last_workgroups));
    TV_HIP(c, hipEventRecord(c->done_ev[buf], c->stream));
    st.unit++;
    st.row = 0;
    return TV_OK;
}

int stream_end_locked(tv_ctx* c, uint8_t* bitfield_out) {
    StreamState& st = c->st;
    if (!st.active) return fail(c, TV_ERR_STATE, "tv_stream_begin has not been called");
    if (st.outstanding || st.unit < st.nunits) {
        const unsigned long long done = st.unit, all = st.nunits;
        stream_abort_locked(c);
        return fail(c, TV_ERR_STATE, "stream ended before its last column (%llu of %llu hashed); aborted", done, all);
    }
    if (c->count) {
        if (!bitfield_out) {
            stream_abort_locked(c);
            return fail(c, TV_ERR_ARG, "bitfield_out is NULL");
        }
        TV_HIP(c, hipEventRecord(c->ev_k1, c->stream));
        int rc = read_bits(c, bitfield_out);
        if (rc) {
            stream_abort_locked(c);
            return rc;
        }
        for (size_t k = 0; k < st.av.size(); k++) bitfield_out[k] &= st.av[k];  // unreadable pieces: bit 0
        c->last_kernel = st.kernel;
        c->last_launches = (int)st.nunits;
        rc = finish_timing(c);
        st = StreamState{};
        return rc;
    }
    st = StreamState{};
    return TV_OK;
}


// Public stream calls: a HIP failure leaves the stream unusable, so it is aborted (the ctx stays usable).
int stream_result(tv_ctx* c, int rc) {
    if (rc == TV_ERR_HIP || rc == TV_ERR_NOMEM) stream_abort_locked(c);
    return rc;
}


}  // namespace tvi

using namespace tvi;

extern "C" {

// End-to-end verification from a host buffer holding the whole shard (tv_verify_host): the stream engine
// with the caller's buffer as the producer.  Each request's rows are one 2D DMA straight from a page-locked
// source (src pitch L) or are gathered into the request's ring slot first.  Rows past src_len are not
// copied; their pieces are unreadable.
int tv_verify_host(tv_ctx* c, const uint8_t* src, uint64_t src_len, const uint8_t* avail_bits,
                   uint8_t* bitfield_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, true);
    if (rc) return rc;
    if (!bitfield_out && c->count) return fail(c, TV_ERR_ARG, "bitfield_out is NULL");
    if (!src && src_len) return fail(c, TV_ERR_ARG, "src is NULL");
    if (!c->count) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    // pieces whose bytes extend past src_len are unreadable
    std::vector<uint8_t> av((c->count + 7) / 8, 0);
    for (uint64_t j = 0; j < c->count; j++) {
        const uint64_t end = j * c->L + piece_len(c, c->first + j);
        if (end <= src_len && (!avail_bits || get_bit(avail_bits, j))) set_bit(av.data(), j);
    }
    const bool pinned = is_pinned(src);
    uint64_t col = 0, win = 0;   // windows x columns within the device budget (or 1 GiB), unless a width is set
    if (!c->stream_chunk && !stream_rows(c))
        budget_geometry(c, c->budget_opt ? c->budget_opt : (1ull << 30), 2048, &col, &win);
    DrainGuard drain(c);  // no DMA reads the caller's buffer after the call returns, also on error paths
    rc = stream_begin_locked(c, av.data(), col, win);
    if (rc) {
        stream_abort_locked(c);
        return rc;
    }
    for (;;) {
        tv_stream_req req;
        rc = stream_next_locked(c, &req);
        if (rc || !req.rows) break;
        // rows wholly inside src: a prefix of the request (its rows ascend in linear offset)
        const uint64_t base = (req.piece - c->first) * c->L + req.offset;
        uint64_t k = 0;
        while (k < req.rows && base + k * c->L + row_bytes(c, req.piece + k, req.offset, req.width) <= src_len) k++;
        rc = stream_commit_locked(c, &req, k ? src + base : nullptr, c->L, pinned, k);
        if (rc) break;
    }
    if (rc) {
        stream_abort_locked(c);
        return rc;
    }
    return stream_end_locked(c, bitfield_out);
}

// The resume check from FILES through the bounded ring (tv_stream_file_table): the stream engine with the library's
// own readers as the producer.  Each request's rows (bytes [offset, offset + width) of consecutive pieces: a column
// across the shard) are read by the lane-0 pool straight from the files into the request's ring slot, each row's
// linear range walked over the file table as Storage.get walks it (storage.ts:98-137); the kernels hash one column
// while the next is read.  Device memory: two columns (TV_OPT_STREAM_CHUNK bytes of every shard piece), so a shard
// verifies under a small device budget with every piece's SHA-1 advancing at once, where windows of whole pieces
// pay one piece's serial SHA-1 per window.  A piece is unreadable exactly when fsStorage.get would return null
// for it: a byte of it in a missing, unopenable or too-short file, a zero-length segment of its walk whose open
// fails (storage.ts:109-110,158), or bytes past the files' end.  Files are opened as fsStorage.get opens them
// (TV_OPT_OPEN_RW), kept open for the call, never created.
int tv_stream_file_table(tv_ctx* c, uint64_t n, const uint64_t* lengths, const char* paths, uint64_t paths_bytes,
                         const uint8_t* avail_bits, uint8_t* bitfield_out, int32_t* status_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, true);
    if (rc) return rc;
    if (!bitfield_out && c->count) return fail(c, TV_ERR_ARG, "bitfield_out is NULL");
    if (n && (!lengths || !paths || !status_out)) return fail(c, TV_ERR_ARG, "NULL argument");
    std::vector<const char*> path(n);
    std::vector<uint64_t> start(n + 1, 0);   // file k's linear bytes: [start[k], start[k + 1])
    for (uint64_t k = 0, o = 0; k < n; k++) {
        const void* z = o < paths_bytes ? memchr(paths + o, 0, paths_bytes - o) : nullptr;
        if (!z)
            return fail(c, TV_ERR_ARG, "paths holds %llu NUL-terminated paths in %llu bytes, the table %llu files",
                        (unsigned long long)k, (unsigned long long)paths_bytes, (unsigned long long)n);
        path[k] = paths + o;
        o = (uint64_t)((const char*)z - paths) + 1;
        if (lengths[k] > UINT64_MAX - start[k])
            return fail(c, TV_ERR_ARG, "file %llu: the lengths overflow 64-bit offsets", (unsigned long long)k);
        start[k + 1] = start[k] + lengths[k];
        status_out[k] = TV_OK;
    }
    if (!c->count) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    const uint64_t last = c->first + c->count - 1;
    const uint64_t lo = c->first * c->L, hi = std::min(c->total, last * c->L + piece_len(c, last));
    // Whether the shard's files are mostly not in the page cache (TV_OPT_FILE_ODIRECT): up to 16 of the files holding
    // >= 1 MiB of its bytes, evenly spread, each sampled as the staging path samples a unit (64 pages), weighted by
    // bytes.  A cold shard is read in longer rows (fewer pieces per window) by more readers: O_DIRECT reads wait on
    // the disk, which wants long requests and many in flight (profiles/r06/window_bench_cold_cols*.jsonl).
    bool cold = false;
    if (c->file_odirect) {
        std::vector<uint64_t> big;
        for (uint64_t k = 0; k < n; k++) {
            const uint64_t a = std::max(lo, start[k]), b = std::min(hi, start[k + 1]);
            if (b > a && b - a >= (1u << 20) && path[k][0]) big.push_back(k);
        }
        double hit = 0, all = 0;
        const size_t m = std::min<size_t>(16, big.size());
        for (size_t q = 0; q < m; q++) {
            const uint64_t k = big[q * big.size() / m];
            const uint64_t a = std::max(lo, start[k]), b = std::min(hi, start[k + 1]);
            // (nonblocking: a FIFO in the table must not hang the sample; only regular files are sampled)
            const int fd = open(path[k], O_RDONLY | O_NONBLOCK | O_CLOEXEC);
            if (fd < 0) continue;
            struct stat sb;
            const double f = fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode) ? cached_fraction(fd, a - start[k], b - a) : -1;
            close(fd);
            if (f < 0) continue;
            hit += f * (double)(b - a);
            all += (double)(b - a);
        }
        cold = all > 0 && hit < 0.5 * all;
    }
    // Geometry: windows x columns within the budget (TV_OPT_RESIDENT_BUDGET, or 1 GiB); a cold shard's windows are
    // 512 pieces (rows 4 x longer; ~44 GB/s of hashing, above what the disk gives).  An explicit TV_OPT_STREAM_CHUNK
    // keeps the engine's columns across the whole shard.
    uint64_t col = 0, win = 0;
    if (!c->stream_chunk) {
        const uint64_t min_win = cold ? (c->stream_cold_window ? c->stream_cold_window : 512) : 2048;
        budget_geometry(c, c->budget_opt ? c->budget_opt : (1ull << 30), min_win, &col, &win);
    }
    // availability before any read: the caller's bits, pieces past the files' end, and the pieces whose walk has a
    // zero-length segment whose open fails (the same segments tv_stage_file_table checks)
    std::vector<uint8_t> av((c->count + 7) / 8, 0);
    for (uint64_t j = 0; j < c->count; j++) {
        const uint64_t i = c->first + j, end = i * c->L + piece_len(c, i);
        if (end <= std::min(c->total, start[n]) && (!avail_bits || get_bit(avail_bits, j))) set_bit(av.data(), j);
    }
    {
        std::vector<TableSeg> segs;
        uint64_t bad = 0, reached = 0;
        if (!walk_file_table(n, lengths, lo, hi, c->L, &segs, &bad, &reached))
            return fail(c, TV_ERR_ARG, "file %llu: the lengths overflow 64-bit offsets", (unsigned long long)bad);
        for (const TableSeg& sg : segs) {
            if (sg.len || sg.linear < lo || sg.linear >= hi) continue;
            if (fs_openable(path[sg.file], c->open_rw)) {
                status_out[sg.file] = TV_ERR_IO;
                const uint64_t j = sg.linear / c->L - c->first;
                av[j >> 3] &= (uint8_t)~(0x80u >> (j & 7));
            }
        }
    }
    // the call's open files: the first kCachedFds opened stay open until the end (a one- or few-file torrent opens
    // each once); past that a reader opens and closes the file around its read (as fsStorage.get does per call), so
    // a 10,000-file torrent never runs into the descriptor limit.  -2: the open failed.  A cached file whose pages
    // are mostly not in the page cache at its open (64 sampled pages, TV_OPT_FILE_ODIRECT) is also opened O_DIRECT:
    // its rows are read past the page cache (dfds; -1 none, and a file whose O_DIRECT read the filesystem refuses
    // reads buffered from then on: no_direct).
    constexpr int kCachedFds = 256;
    std::vector<int> fds(n, -1), dfds(n, -1);
    std::unique_ptr<std::atomic<bool>[]> no_direct(new std::atomic<bool>[n ? n : 1]());
    int cached = 0;
    std::mutex fd_mu;
    struct Closer {
        std::vector<int>& f;
        std::vector<int>& d;
        ~Closer() {
            for (int x : f)
                if (x >= 0) close(x);
            for (int x : d)
                if (x >= 0) close(x);
        }
    } closer{fds, dfds};
    // -> a descriptor of file k, and whether the caller closes it after its read; *dfd: its O_DIRECT one or -1
    auto fd_of = [&](uint64_t k, bool* own, int* dfd) -> int {
        *own = false;
        *dfd = -1;
        {
            std::lock_guard<std::mutex> fg(fd_mu);
            if (fds[k] != -1) {
                if (dfds[k] >= 0 && !no_direct[k].load(std::memory_order_relaxed)) *dfd = dfds[k];
                return fds[k];
            }
        }
        int e = 0;
        const int d = path[k][0] ? open_file(path[k], c->open_rw, &e) : -1;
        std::lock_guard<std::mutex> fg(fd_mu);
        if (fds[k] != -1) {   // another reader opened it meanwhile
            if (d >= 0) close(d);
            if (dfds[k] >= 0 && !no_direct[k].load(std::memory_order_relaxed)) *dfd = dfds[k];
            return fds[k];
        }
        if (d < 0) {
            if (e != EMFILE && e != ENFILE) fds[k] = -2;   // (out of descriptors: not the file's failure, but unread)
            return -1;
        }
        if (cached < kCachedFds) {
            cached++;
            fds[k] = d;
            if (c->file_odirect && lengths[k] >= (1u << 20)) {
                const double f = cached_fraction(d, 0, lengths[k]);
                if (f >= 0 && f < 0.5) dfds[k] = open(path[k], (c->open_rw ? O_RDWR : O_RDONLY) | O_DIRECT | O_CLOEXEC);
                if (dfds[k] >= 0) *dfd = dfds[k];
            }
            return d;
        }
        *own = true;
        return d;
    };
    // file bytes [fo, fo + len) -> dst through the O_DIRECT descriptor: straight into dst when the file offset, dst
    // and the length are 4 KiB-aligned (whole-row reads of a one-file torrent), else via a 4 KiB-aligned scratch of
    // the reader thread's in 4 MiB steps.  -> bytes read (short: the file ended), or -errno.
    auto read_direct = [&](int dfd, uint64_t fo, uint8_t* dst, uint64_t len) -> int64_t {
        if (c->file_odirect == 2) return -EINVAL;   // (fault injection: the filesystem refusing O_DIRECT reads)
        uint64_t o = 0;
        if (fo % 4096 == 0 && (uintptr_t)dst % 4096 == 0 && len % 4096 == 0) {
            while (o < len) {
                const ssize_t got = pread(dfd, dst + o, len - o, (off_t)(fo + o));
                if (got < 0 && errno == EINTR) continue;
                if (got < 0) return -errno;
                if (got == 0) break;
                o += (uint64_t)got;
            }
            return (int64_t)o;
        }
        constexpr uint64_t kStep = 4ull << 20;
        struct Scratch {   // (sized to the longest read the thread has needed: a row, at most kStep + 8 KiB)
            uint8_t* p = nullptr;
            uint64_t cap = 0;
            ~Scratch() { free(p); }
        };
        thread_local Scratch scratch;
        const uint64_t need = std::min(kStep, len) + 8192;
        if (scratch.cap < need) {
            free(scratch.p);
            scratch.cap = 0;
            if (posix_memalign((void**)&scratch.p, 4096, need)) {
                scratch.p = nullptr;
                return -ENOMEM;
            }
            scratch.cap = need;
        }
        while (o < len) {
            const uint64_t at = fo + o, al = at / 4096 * 4096, lead = at - al;
            const uint64_t m = std::min(kStep, len - o), ask = (lead + m + 4095) / 4096 * 4096;
            uint64_t got_all = 0;
            while (got_all < ask) {
                const ssize_t got = pread(dfd, scratch.p + got_all, ask - got_all, (off_t)(al + got_all));
                if (got < 0 && errno == EINTR) continue;
                if (got < 0) return -errno;
                if (got == 0) break;
                got_all += (uint64_t)got;
            }
            const uint64_t have = got_all > lead ? std::min(m, got_all - lead) : 0;
            memcpy(dst + o, scratch.p + lead, have);
            o += have;
            if (have < m) break;   // the file ended
        }
        return (int64_t)o;
    };
    const int readers = cold ? (c->stream_cold_readers ? c->stream_cold_readers : 2 * c->file_threads) : c->file_threads;
    DrainGuard drain(c);  // (the ring's copies and the column kernels are done when the call returns)
    rc = stream_begin_locked(c, av.data(), col, win, cold ? c->stream_cold_req : 0);
    if (rc) {
        stream_abort_locked(c);
        return rc;
    }
    std::vector<std::atomic<int32_t>> file_err(n);
    for (auto& e : file_err) e.store(TV_OK);
    for (;;) {
        tv_stream_req req;
        rc = stream_next_locked(c, &req);
        if (rc || !req.rows) break;
        uint8_t* slot = c->ring[c->st.slot];
        std::vector<uint8_t> row_bad(req.rows, 0);
        c->pool[0].run(readers, req.rows, [&](uint64_t q) {
            const uint64_t i = req.piece + q, j = i - c->first;
            const uint64_t nb = row_bytes(c, i, req.offset, req.width);
            if (!nb || !get_bit(c->st.av.data(), j)) return;
            const uint64_t a = i * c->L + req.offset, b = a + nb;   // the row's linear bytes
            uint8_t* out = slot + q * req.width;
            // the file holding byte a: the last k with start[k] <= a < start[k + 1] (zero-length files skipped)
            uint64_t k = (uint64_t)(std::upper_bound(start.begin(), start.end(), a) - start.begin()) - 1;
            for (uint64_t pos = a; pos < b && k < n; k++) {
                if (start[k + 1] <= pos) continue;
                const uint64_t e = std::min(b, start[k + 1]);
                bool own = false;
                int dfd = -1;
                const int fd = fd_of(k, &own, &dfd);
                uint64_t o = 0;
                if (dfd >= 0) {
                    const int64_t got = read_direct(dfd, pos - start[k], out + (pos - a), e - pos);
                    if (got >= 0) {
                        o = (uint64_t)got;
                        c->file_ns[TV_FILE_BYTES_ODIRECT].fetch_add(o, std::memory_order_relaxed);
                    } else {
                        // an O_DIRECT read the filesystem refuses is not the file's failure: this file reads buffered
                        // from here on, this row included (counted, first errno kept, as the staging path's fallback)
                        no_direct[k].store(true, std::memory_order_relaxed);
                        c->file_ns[TV_FILE_ODIRECT_FALLBACKS].fetch_add(1, std::memory_order_relaxed);
                        uint64_t none = 0;
                        c->file_ns[TV_FILE_ODIRECT_ERRNO].compare_exchange_strong(none, (uint64_t)-got);
                    }
                }
                while (fd >= 0 && o < e - pos) {
                    const ssize_t got = pread(fd, out + (pos - a) + o, e - pos - o, (off_t)(pos - start[k] + o));
                    if (got < 0 && errno == EINTR) continue;
                    if (got <= 0) break;
                    o += (uint64_t)got;
                }
                if (own) close(fd);
                c->file_ns[TV_FILE_BYTES_READ].fetch_add(o, std::memory_order_relaxed);
                if (o < e - pos) {   // missing, unopenable or short: the piece is null, as fsStorage.get's read
                    row_bad[q] = 1;
                    file_err[k].store(TV_ERR_IO);
                    return;
                }
                pos = e;
            }
        });
        for (uint64_t q = 0; q < req.rows; q++) {
            if (!row_bad[q]) continue;
            const uint64_t j = req.piece + q - c->first;
            c->st.av[j >> 3] &= (uint8_t)~(0x80u >> (j & 7));
        }
        rc = stream_commit_locked(c, &req, nullptr, 0, true, req.rows);
        if (rc) break;
    }
    for (uint64_t k = 0; k < n; k++)
        if (file_err[k].load() != TV_OK) status_out[k] = TV_ERR_IO;
    if (rc) {
        stream_abort_locked(c);
        return rc;
    }
    return stream_end_locked(c, bitfield_out);
}

int tv_stream_begin(tv_ctx* c, const uint8_t* avail_bits) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, true);
    if (rc) return rc;
    TV_HIP(c, hipSetDevice(c->device));
    return stream_result(c, stream_begin_locked(c, avail_bits));
}

int tv_stream_next(tv_ctx* c, tv_stream_req* req) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    if (!req) return fail(c, TV_ERR_ARG, "req is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    TV_HIP(c, hipSetDevice(c->device));
    return stream_result(c, stream_next_locked(c, req));
}

int tv_stream_commit(tv_ctx* c, const tv_stream_req* req) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    TV_HIP(c, hipSetDevice(c->device));
    return stream_result(c, stream_commit_locked(c, req, nullptr, 0, true, req ? req->rows : 0));
}

int tv_stream_commit_from(tv_ctx* c, const tv_stream_req* req, const uint8_t* src, uint64_t src_pitch) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    if (!src) return fail(c, TV_ERR_ARG, "src is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (req && req->rows > 1 && src_pitch < req->width)
        return fail(c, TV_ERR_ARG, "src_pitch %llu is shorter than the row width %llu", (unsigned long long)src_pitch,
                    (unsigned long long)req->width);
    TV_HIP(c, hipSetDevice(c->device));
    return stream_result(c, stream_commit_locked(c, req, src, src_pitch, is_pinned(src), req ? req->rows : 0));
}

int tv_stream_unreadable(tv_ctx* c, uint64_t piece) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->st.active) return fail(c, TV_ERR_STATE, "tv_stream_begin has not been called");
    if (piece < c->first || piece >= c->first + c->count)
        return fail(c, TV_ERR_ARG, "piece %llu is not in this context's shard", (unsigned long long)piece);
    const uint64_t j = piece - c->first;
    c->st.av[j >> 3] &= (uint8_t)~(0x80u >> (j & 7));
    return TV_OK;
}

int tv_stream_end(tv_ctx* c, uint8_t* bitfield_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    TV_HIP(c, hipSetDevice(c->device));
    return stream_end_locked(c, bitfield_out);
}

int tv_stream_abort(tv_ctx* c) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    TV_HIP(c, hipSetDevice(c->device));
    stream_abort_locked(c);
    return TV_OK;
}

int tv_stream_fill_synthetic(tv_ctx* c, const tv_stream_req* req, uint64_t seed) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    const StreamState& st = c->st;
    if (!st.active || !st.outstanding) return fail(c, TV_ERR_STATE, "no outstanding request (call tv_stream_next)");
    if (!req || req->seq != st.req.seq) return fail(c, TV_ERR_ARG, "the request does not match the outstanding one");
    const tv_stream_req r = st.req;
    uint8_t* slot = c->ring[st.slot];
    c->pool[0].run(c->file_threads, r.rows, [&](uint64_t q) {
        const uint64_t i = r.piece + q;
        tv_synth_fill_host(seed, i * c->L + r.offset, row_bytes(c, i, r.offset, r.width), slot + q * r.width);
    });
    return TV_OK;
}

}  // extern "C"
