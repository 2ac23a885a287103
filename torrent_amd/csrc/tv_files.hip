// tv_files.hip -- staging from files (tv_stage_file, tv_stage_files): the reference's fsStorage.get reads
// (storage.ts:149-172) done by the library's own threads, segment by segment as Storage.get's walk maps them
// (storage.ts:89-137), with the reference's failure rules (a null piece, never an error) decided here.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "tv_ctx.h"

using namespace tvi;

namespace {

#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22  // Linux >= 5.14; older kernels fall back to touching every page
#endif

// Fault in the pages of a mapped file window [m, m + n) (the MAP_POPULATE equivalent, after the
// residency check).  One thread: splitting it over 8 was 27 % slower on a warm page cache (mm lock
// contention; tools/stage_file_bench.py, profiles/r01/stage_file_bench.log).
void populate_window(void* m, uint64_t n) {
    if (madvise(m, n, MADV_POPULATE_READ) == 0) return;
    volatile uint8_t sink = 0;
    for (uint64_t o = 0; o < n; o += 4096) sink = sink ^ ((const uint8_t*)m)[o];
    (void)sink;
}

// Fraction of the pages of the mapped window [m, m + n) that are in the page cache (mincore).
double resident_fraction(void* m, uint64_t n, uint64_t page) {
    std::vector<unsigned char> vec((n + page - 1) / page);
    if (mincore(m, n, vec.data()) != 0) return 0.0;
    size_t r = 0;
    for (unsigned char v : vec) r += v & 1;
    return vec.empty() ? 1.0 : (double)r / (double)vec.size();
}

// Read file bytes [fo, fo + n) into dst with parallel preads (4 MiB parts on up to max_threads threads,
// TV_OPT_FILE_THREADS: a cold file is read with many large requests in flight).  Returns 0 or an
// errno value (EIO for a short read).
int pread_parallel(int fd, uint8_t* dst, uint64_t fo, uint64_t n, int max_threads, const cpu_set_t* cpus) {
    const uint64_t part = 4ull << 20;
    const uint64_t nparts = (n + part - 1) / part;
    const int threads = (int)std::min<uint64_t>((uint64_t)std::max(1, max_threads), nparts);
    std::vector<int> err(threads, 0);
    auto work = [&](int t) {
        for (uint64_t q = t; q < nparts; q += threads) {
            uint64_t o = q * part;
            const uint64_t e = std::min(n, o + part);
            while (o < e) {
                const ssize_t got = pread(fd, dst + o, e - o, (off_t)(fo + o));
                if (got < 0 && errno == EINTR) continue;
                if (got <= 0) {
                    err[t] = got < 0 ? errno : EIO;
                    return;
                }
                o += (uint64_t)got;
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++)
        th.emplace_back([&work, cpus, t] {
            pin_thread(cpus);
            work(t);
        });
    if (threads > 0) work(0);
    for (auto& t : th) t.join();
    for (int e : err)
        if (e) return e;
    return 0;
}

// Memory-mapped windows of a file for tv_stage_file; released (unregistered, unmapped) on every exit.
// Declared BEFORE the call's DrainGuard, so the streams are drained before any window goes away.
struct FileWindows {
    struct W {
        void* ptr = nullptr;
        size_t len = 0;
        bool registered = false;
    };
    W w[2];
    int fd = -1;
    void release(int k) {
        if (w[k].registered) (void)hipHostUnregister(w[k].ptr);
        if (w[k].ptr) munmap(w[k].ptr, w[k].len);
        w[k] = W{};
        (void)hipGetLastError();
    }
    ~FileWindows() {
        release(0);
        release(1);
        if (fd >= 0) close(fd);
    }
};


// tv_stage_file with the context lock held and the arguments checked.
int stage_file_locked(tv_ctx* c, const char* path, uint64_t file_offset, uint64_t linear_offset, uint64_t len,
                      int lane = 0) {
    hipStream_t cs = lane_stream(c, lane);
    int rc = TV_OK;
    if (len == 0) {  // reads nothing, but fsStorage.get still opens the path (storage.ts:158)
        const int e = fs_openable(path, c->open_rw);
        return e ? fail(c, TV_ERR_IO, "open %s: %s", path, strerror(e)) : TV_OK;
    }
    FileWindows win;  // before `drain`: destroyed after the streams are drained
    int oe = 0;
    win.fd = open_file(path, c->open_rw, &oe);
    if (win.fd < 0)
        return fail(c, TV_ERR_IO, "open %s for %s: %s", path, c->open_rw ? "read and write" : "reading", strerror(oe));
    struct stat st;
    if (fstat(win.fd, &st) != 0) return fail(c, TV_ERR_IO, "fstat %s: %s", path, strerror(errno));
    if ((uint64_t)st.st_size < file_offset + len)
        return fail(c, TV_ERR_IO, "%s has %llu bytes, the read needs %llu", path, (unsigned long long)st.st_size,
                    (unsigned long long)(file_offset + len));
    if (c->count == 0) return TV_OK;
    uint64_t a, b;
    clip_to_shard(c, linear_offset, len, &a, &b);
    if (a >= b) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    DrainGuard drain(c, lane, /*sync_compute=*/false);
    for (int k = 0; k < 2; k++) TV_HIP(c, hipEventCreateWithFlags(&drain.ev[k], hipEventDisableTiming));
    const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
    const uint64_t chunk = c->file_chunk;
    int idx = 0;
    for (uint64_t p = a; p < b; p += chunk, idx++) {
        const int k = idx & 1;
        const uint64_t n = std::min(chunk, b - p);
        const uint64_t fo = file_offset + (p - linear_offset);
        // the window used two chunks ago must be DMA-complete before it is unmapped
        if (win.w[k].ptr) {
            TV_HIP(c, hipEventSynchronize(drain.ev[k]));
            win.release(k);
        }
        const uint64_t map_off = fo / page * page, delta = fo - map_off;
        // (a file that cannot be mapped, e.g. on a filesystem without mmap, takes the pread path)
        void* m = c->file_direct ? mmap(nullptr, delta + n, PROT_READ, MAP_SHARED, win.fd, (off_t)map_off) : MAP_FAILED;
        if (m != MAP_FAILED) {
            win.w[k].ptr = m;
            win.w[k].len = delta + n;
        }
        // direct only when the file bytes and the resident bytes agree mod 4 (else the DMA is unaligned)
        if (m != MAP_FAILED && ((fo ^ p) & 3) == 0 && resident_fraction(m, delta + n, page) >= 0.5) {
            // warm window: register its page-cache pages read-only and DMA them to HBM directly
            populate_window(m, delta + n);
            win.w[k].registered = hipHostRegister(m, delta + n, hipHostRegisterReadOnly) == hipSuccess;
            (void)hipGetLastError();
        }
        if (win.w[k].registered) {
            rc = stage_range(c, p, p + n, (const uint8_t*)m + delta, p, true, lane);
            if (rc) return rc;
        } else {
            // cold window (or direct DMA off / refused): parallel preads into the pinned ring, then DMA
            win.release(k);
            for (uint64_t q = 0; q < n; q += kRingSlotBytes - 4) {
                const uint64_t kq = std::min<uint64_t>(kRingSlotBytes - 4, n - q);
                SlotLease slot(c, lane);  // lent until every copy out of it is queued
                rc = slot.take();
                if (rc) return rc;
                uint8_t* at = slot.ptr() + ((p + q) & 3);  // at the resident bytes' alignment mod 4
                const int e = pread_parallel(win.fd, at, fo + q, kq, c->file_threads, numa_cpus(c));
                if (e) return fail(c, TV_ERR_IO, "read %s at %llu: %s", path, (unsigned long long)(fo + q), strerror(e));
                rc = stage_range(c, p + q, p + q + kq, at, p + q, true, lane, /*src_in_ring=*/true);
                if (rc) return rc;
                rc = slot.release();
                if (rc) return rc;
            }
        }
        TV_HIP(c, hipEventRecord(drain.ev[k], cs));
    }
    TV_HIP(c, hipStreamSynchronize(cs));
    return TV_OK;
}

// Read every segment of `segs` into slot memory at its packed offset, on `threads` threads (each
// segment: open, pread loop, close).  A missing, unreadable or short file sets its status to TV_ERR_IO.
struct SmallSeg {
    uint64_t k, file_offset, linear, len, packed;
};

void read_segments(Pool& pool, const std::vector<SmallSeg>& segs, size_t lo, size_t hi, const char* const* paths,
                   uint8_t* slot, int32_t* status, int threads, bool rw, std::string* first_err, std::mutex* err_mu) {
    // work items: (segment, part) with parts of at most 4 MiB, so one long segment is read by many threads;
    // run on the lane's persistent workers (a thread spawn per 64 MiB slot cost ~15 x 20-50 us per slot)
    constexpr uint64_t kPart = 4ull << 20;
    std::vector<std::pair<size_t, uint64_t>> items;
    for (size_t q = lo; q < hi; q++)
        for (uint64_t o = 0; o < segs[q].len; o += kPart) items.emplace_back(q, o);
    pool.run(threads, items.size(), [&](uint64_t it) {
        const SmallSeg& sg = segs[items[it].first];
        const uint64_t part0 = items[it].second, part1 = std::min(sg.len, part0 + kPart);
        const char* path = paths[sg.k];
        int e = 0;
        const int fd = open_file(path, rw, &e);  // as fsStorage.get opens it, read + write (storage.ts:28-32)
        if (fd >= 0) {
            uint64_t o = part0;
            while (o < part1) {
                const ssize_t got = pread(fd, slot + sg.packed + o, part1 - o, (off_t)(sg.file_offset + o));
                if (got < 0 && errno == EINTR) continue;
                if (got <= 0) {
                    e = got < 0 ? errno : EIO;  // 0 bytes: the file is shorter than the segment
                    break;
                }
                o += (uint64_t)got;
            }
            close(fd);
        }
        if (e) {
            status[sg.k] = TV_ERR_IO;
            std::lock_guard<std::mutex> g(*err_mu);
            if (first_err->empty()) *first_err = std::string(path) + ": " + strerror(e);
        }
    });
}

// Mark the shard pieces holding linear bytes [a, b) unreadable (tv_verify reports them 0).
void mark_bad(tv_ctx* c, uint64_t a, uint64_t b) {
    const uint64_t lo = c->first * c->L;
    const uint64_t last = c->first + c->count - 1;
    const uint64_t hi = last * c->L + piece_len(c, last);
    if (a == b) {  // a zero-length segment: the piece it sits in
        if (a < lo || a >= hi) return;
        b = a + 1;
    }
    a = std::max(a, lo);
    b = std::min(b, hi);
    if (a >= b) return;
    for (uint64_t j = a / c->L - c->first; j <= (b - 1) / c->L - c->first; j++) set_bit(c->file_bad.data(), j);
    c->any_file_bad = true;
}

// Bytes of [file_offset, file_offset + len) that fsStorage.get's read of `path` would return: 0 when the
// open (read + write, storage.ts:28-32,158) fails or the path is not a regular file, else what the file holds.
uint64_t readable_prefix(const char* path, uint64_t file_offset, uint64_t len, bool rw) {
    if (access_ok(path, rw)) return 0;
    struct stat st;
    if (stat(path, &st) != 0 || !S_ISREG(st.st_mode)) return 0;
    const uint64_t size = (uint64_t)st.st_size;
    return size <= file_offset ? 0 : std::min(len, size - file_offset);
}

// A file segment staging could not read whole: Storage.get reads per piece (storage.ts:50-65), so the
// pieces inside the file's readable prefix are still readable.  Stage that prefix again and mark the pieces
// from the first missing byte to the segment's end unreadable (a zero-length segment: its piece).
int recover_segment(tv_ctx* c, const char* path, uint64_t file_offset, uint64_t linear_offset, uint64_t len) {
    if (len == 0) {
        mark_bad(c, linear_offset, linear_offset);
        return TV_OK;
    }
    uint64_t r = readable_prefix(path, file_offset, len, c->open_rw);
    if (r == len) r = 0;  // readable by size yet the read failed (an I/O error): nothing of it counts
    // only the prefix's whole pieces are staged: the piece holding its first missing byte is marked below
    const uint64_t whole = (linear_offset + r) / c->L * c->L;
    r = whole > linear_offset ? whole - linear_offset : 0;
    if (r) {
        const int rc = stage_file_locked(c, path, file_offset, linear_offset, r);
        if (rc == TV_ERR_IO) r = 0;
        else if (rc) return rc;
    }
    mark_bad(c, linear_offset + r, linear_offset + len);
    return TV_OK;
}

}  // namespace

extern "C" {

int tv_stage_file(tv_ctx* c, const char* path, uint64_t file_offset, uint64_t linear_offset, uint64_t len) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (!path) return fail(c, TV_ERR_ARG, "path is NULL");
    if (linear_offset + len < linear_offset || file_offset + len < file_offset)
        return fail(c, TV_ERR_ARG, "offset + len overflows");
    uint64_t a = 0, b = 0;
    if (c->count) clip_to_whole_shard(c, linear_offset, len, &a, &b);
    if (!c->win || len == 0 || a >= b) {
        rc = stage_file_locked(c, path, file_offset, linear_offset, len);
        if (rc == TV_OK) clear_bad(c, a, b);
        if (rc != TV_ERR_IO || c->count == 0) return rc;
        const std::string err = c->err;
        const int r = recover_segment(c, path, file_offset, linear_offset, len);
        if (r) return r;
        fail(c, TV_ERR_IO, "%s", err.c_str());  // the first failure stays the call's message
        return TV_ERR_IO;
    }
    // windowed layout: the segment window by window (each part is checked, staged and recovered on its own, so a
    // short file still keeps its whole pieces before the first missing byte)
    TV_HIP(c, hipSetDevice(c->device));
    std::string first_err;
    for (uint64_t pos = a; pos < b;) {
        const uint64_t w = win_of(c, pos / c->L - c->first);
        rc = win_enter(c, w);
        if (rc) return rc;
        const uint64_t e = std::min(b, win_end_linear(c, w));
        const uint64_t fo = file_offset + (pos - linear_offset);
        rc = stage_file_locked(c, path, fo, pos, e - pos);
        if (rc == TV_OK) {
            clear_bad(c, pos, e);
        } else if (rc == TV_ERR_IO) {
            if (first_err.empty()) first_err = c->err;
            rc = recover_segment(c, path, fo, pos, e - pos);
            if (rc) return rc;
        } else {
            return rc;
        }
        pos = e;
    }
    if (first_err.empty()) return TV_OK;
    fail(c, TV_ERR_IO, "%s", first_err.c_str());
    return TV_ERR_IO;
}

}  // extern "C"

namespace {

// tv_stage_files with the lock held and the arguments checked: every segment's bytes among the resident pieces
// (clip_to_shard: the shard, or a windowed layout's open window).  status_out[k] is set to TV_ERR_IO on a
// failure and left alone otherwise.  check_zero: check the zero-length segments' opens (once per call).
int stage_files_core(tv_ctx* c, uint64_t n, const char* const* paths, const uint64_t* file_offsets,
                     const uint64_t* linear_offsets, const uint64_t* lens, int32_t* status_out, bool check_zero) {
    int rc = TV_OK;
    // Long segments: the windowed page-cache path of tv_stage_file.  Short ones: packed into the pinned
    // ring's 64 MiB slots, read by the thread pool, DMA'd per run of linear-contiguous segments while the
    // next slot is read.  With TV_OPT_FILE_CONCURRENT the long segments are split by bytes between a
    // helper thread on staging lane 1 and this thread (lane 0, before the pool): each lane's copies
    // queue on its own stream, so the two feed the DMA engines side by side.
    const uint64_t direct_min = c->file_direct_min;
    struct LongSeg {
        uint64_t k, fo, a, len;
    };
    std::vector<LongSeg> longs;
    std::vector<SmallSeg> small;
    uint64_t small_bytes = 0;
    std::string zero_err;
    for (uint64_t k = 0; k < n; k++) {
        if (lens[k] == 0) {  // Storage.get's zero-length segments: only the open decides (storage.ts:109-110,158)
            if (!check_zero) continue;
            if (const int e = fs_openable(paths[k], c->open_rw)) {
                status_out[k] = TV_ERR_IO;
                if (zero_err.empty()) zero_err = std::string(paths[k]) + ": " + strerror(e);
            }
            continue;
        }
        uint64_t a, b;
        clip_to_shard(c, linear_offsets[k], lens[k], &a, &b);
        if (a >= b) continue;  // nothing of this segment is resident here
        const uint64_t fo = file_offsets[k] + (a - linear_offsets[k]);
        if (b - a >= direct_min) {
            longs.push_back({k, fo, a, b - a});
        } else {
            const uint64_t part = kRingSlotBytes - 4;  // (pieces of at most one slot, with room to align)
            for (uint64_t o = 0; o < b - a; o += part)
                small.push_back({k, fo + o, a + o, std::min<uint64_t>(part, b - a - o), 0});
            small_bytes += b - a;
        }
    }
    // longest first to the lane with fewer bytes so far (lane 0 also carries the pool's bytes)
    std::vector<LongSeg> lane_segs[2];
    {
        std::vector<size_t> order(longs.size());
        for (size_t q = 0; q < order.size(); q++) order[q] = q;
        std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return longs[x].len > longs[y].len; });
        uint64_t load[2] = {small_bytes, 0};
        for (size_t q : order) {
            const int l = (c->file_concurrent && load[1] < load[0]) ? 1 : 0;
            lane_segs[l].push_back(longs[q]);
            load[l] += longs[q].len;
        }
        for (auto& v : lane_segs)  // each lane walks its segments in linear order
            std::sort(v.begin(), v.end(), [](const LongSeg& x, const LongSeg& y) { return x.a < y.a; });
    }
    int helper_rc = TV_OK;
    std::thread helper;
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{helper};  // every exit joins the helper before the ctx lock is released
    if (!lane_segs[1].empty()) {
        helper = std::thread([&]() {
            pin_thread(numa_cpus(c));  // next to its ring and the GPU (TV_OPT_NUMA_BIND)
            if (hipSetDevice(c->device) != hipSuccess) {
                helper_rc = fail(c, TV_ERR_HIP, "tv_stage_files: hipSetDevice(%d) failed", c->device);
                return;
            }
            for (const LongSeg& sg : lane_segs[1]) {
                const int r = stage_file_locked(c, paths[sg.k], sg.fo, sg.a, sg.len, 1);
                if (r == TV_ERR_IO) status_out[sg.k] = TV_ERR_IO;
                else if (r) {
                    helper_rc = r;
                    return;
                }
            }
        });
    }
    for (const LongSeg& sg : lane_segs[0]) {
        rc = stage_file_locked(c, paths[sg.k], sg.fo, sg.a, sg.len, 0);
        if (rc == TV_ERR_IO) status_out[sg.k] = TV_ERR_IO;
        else if (rc) return rc;
    }
    std::string first_err = zero_err;
    std::mutex err_mu;
    DrainGuard drain(c, 0, /*sync_compute=*/false);
    size_t i = 0;
    while (i < small.size()) {
        size_t j = i;
        uint64_t used = 0;
        while (j < small.size()) {
            // each byte sits in the slot at its linear offset's alignment mod 4 (dword-aligned DMA)
            const uint64_t at = used + ((small[j].linear - used) & 3);
            if (at + small[j].len > kRingSlotBytes) break;
            small[j].packed = at;
            used = at + small[j].len;
            j++;
        }
        SlotLease slot(c, 0);  // lent until every copy out of it is queued
        rc = slot.take();
        if (rc) return rc;
        read_segments(c->pool[0], small, i, j, paths, slot.ptr(), status_out, c->file_threads, c->open_rw, &first_err,
                      &err_mu);
        for (size_t q = i; q < j;) {  // one copy per run of readable, linear-contiguous segments
            if (status_out[small[q].k] != TV_OK) { q++; continue; }
            size_t r = q + 1;
            while (r < j && status_out[small[r].k] == TV_OK && small[r].linear == small[r - 1].linear + small[r - 1].len)
                r++;
            const uint64_t lin_a = small[q].linear, lin_b = small[r - 1].linear + small[r - 1].len;
            rc = stage_range(c, lin_a, lin_b, slot.ptr() + small[q].packed, lin_a, true, 0, /*src_in_ring=*/true);
            if (rc) return rc;
            q = r;
        }
        rc = slot.release();
        if (rc) return rc;
        i = j;
    }
    TV_HIP(c, hipStreamSynchronize(c->copy_stream));
    if (helper.joinable()) helper.join();
    if (helper_rc) return helper_rc;
    // the failed segments: their readable prefixes staged again, the rest of their pieces marked unreadable
    for (uint64_t k = 0; k < n; k++) {
        if (status_out[k] != TV_ERR_IO) continue;
        if (lens[k] == 0 && !check_zero) continue;
        rc = recover_segment(c, paths[k], file_offsets[k], linear_offsets[k], lens[k]);
        if (rc) return rc;
    }
    if (!first_err.empty()) fail(c, TV_OK, "tv_stage_files: %s (and possibly more; see status_out)", first_err.c_str());
    return TV_OK;
}

}  // namespace

extern "C" {

int tv_stage_files(tv_ctx* c, uint64_t n, const char* const* paths, const uint64_t* file_offsets,
                   const uint64_t* linear_offsets, const uint64_t* lens, int32_t* status_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (n == 0) return TV_OK;
    if (!paths || !file_offsets || !linear_offsets || !lens || !status_out)
        return fail(c, TV_ERR_ARG, "NULL argument");
    for (uint64_t k = 0; k < n; k++) {
        if (!paths[k]) return fail(c, TV_ERR_ARG, "paths[%llu] is NULL", (unsigned long long)k);
        if (linear_offsets[k] + lens[k] < linear_offsets[k] || file_offsets[k] + lens[k] < file_offsets[k])
            return fail(c, TV_ERR_ARG, "segment %llu: offset + len overflows", (unsigned long long)k);
        status_out[k] = TV_OK;
    }
    if (c->count == 0) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    // the pieces whose every byte this call stages lose an earlier call's unreadable mark (the union of the
    // segments, merged: a piece spanning files is covered by several)
    if (c->any_file_bad) {
        std::vector<std::pair<uint64_t, uint64_t>> iv;
        for (uint64_t k = 0; k < n; k++)
            if (lens[k]) iv.emplace_back(linear_offsets[k], linear_offsets[k] + lens[k]);
        std::sort(iv.begin(), iv.end());
        for (size_t q = 0; q < iv.size();) {
            uint64_t a = iv[q].first, b = iv[q].second;
            size_t r = q + 1;
            for (; r < iv.size() && iv[r].first <= b; r++) b = std::max(b, iv[r].second);
            clear_bad(c, a, b);
            q = r;
        }
    }
    if (!c->win) return stage_files_core(c, n, paths, file_offsets, linear_offsets, lens, status_out, true);
    // windowed layout: the windows the segments touch, ascending; each is staged by one core pass (which skips
    // every byte outside it) and hashed when the next one opens
    const uint64_t nwin = (c->count + c->win_n - 1) / c->win_n;
    std::vector<uint8_t> touched(nwin, 0);
    for (uint64_t k = 0; k < n; k++) {
        uint64_t a, b;
        clip_to_whole_shard(c, linear_offsets[k], lens[k], &a, &b);
        if (a >= b) continue;
        const uint64_t w0 = win_of(c, a / c->L - c->first), w1 = win_of(c, (b - 1) / c->L - c->first);
        std::fill(touched.begin() + (ptrdiff_t)w0, touched.begin() + (ptrdiff_t)w1 + 1, (uint8_t)1);
    }
    bool check_zero = true;  // (the zero-length segments' opens are checked in the first pass)
    for (uint64_t w = 0; w < nwin; w++) {
        if (!touched[w]) continue;
        rc = win_enter(c, w);
        if (!rc) rc = stage_files_core(c, n, paths, file_offsets, linear_offsets, lens, status_out, check_zero);
        if (rc) return rc;
        check_zero = false;
    }
    return check_zero ? stage_files_core(c, n, paths, file_offsets, linear_offsets, lens, status_out, true) : TV_OK;
}

}  // extern "C"
