// tv_files.hip -- staging from files (tv_stage_file, tv_stage_files): the reference's fsStorage.get reads
// (storage.ts:149-172) done by the library's own threads, segment by segment as Storage.get's walk maps them
// (storage.ts:89-137), with the reference's failure rules (a null piece, never an error) decided here.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
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

// Read file bytes [fo, fo + n) into dst with parallel preads on the lane's persistent workers (`threads` of
// them; parts of 1-4 MiB, at least two per thread so the slowest part ends the slot early).  The first `need`
// bytes must all be read (n - need: an O_DIRECT read's rounding past the end of the file, which may come back
// short).  Returns 0 or an errno value (EIO for a short read).  The round-1..4 form spawned `threads` std::threads
// per 64 MiB slot.
int pread_pool(Pool& pool, int threads, int fd, uint8_t* dst, uint64_t fo, uint64_t n, uint64_t need) {
    threads = std::max(1, threads);
    uint64_t part = n / (2 * (uint64_t)threads);
    part = std::min<uint64_t>(4ull << 20, std::max<uint64_t>(1ull << 20, (part + 65535) / 65536 * 65536));
    const uint64_t nparts = (n + part - 1) / part;
    std::atomic<int> err{0};
    pool.run(threads, nparts, [&](uint64_t q) {
        uint64_t o = q * part;
        const uint64_t e = std::min(n, o + part);
        // (o >= need: the bytes asked for are in -- an O_DIRECT read that came back short at the end of the file
        // must not be continued, as its next request would start off a 4 KiB boundary and be refused)
        while (o < e && o < need && !err.load(std::memory_order_relaxed)) {
            const ssize_t got = pread(fd, dst + o, e - o, (off_t)(fo + o));
            if (got < 0 && errno == EINTR) continue;
            if (got <= 0) {
                int expect = 0;
                err.compare_exchange_strong(expect, got < 0 ? errno : EIO);
                return;
            }
            o += (uint64_t)got;
        }
    });
    return err.load();
}

}  // namespace

namespace tvi {

// Fraction of file bytes [fo, fo + n) in the page cache, sampled: the range is mapped (no page is touched) and
// mincore asks for 64 pages spread evenly over it; -1 when it cannot be mapped.  (cachestat(2) would be one call,
// but on an overlay filesystem -- the gpurun boxes' /tmp -- it reports the overlay inode, which caches nothing,
// while mincore sees the pages of the real file the mapping is redirected to: a warm file read as cold there and
// took the O_DIRECT path at disk speed.  A full mincore of a 256 MiB unit costs ~0.9 ms; 64 samples, microseconds.)
double cached_fraction(int fd, uint64_t fo, uint64_t n) {
    if (n == 0) return 1.0;
    const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
    const uint64_t off = fo / page * page, len = (fo - off + n + page - 1) / page * page, npages = len / page;
    void* m = mmap(nullptr, len, PROT_READ, MAP_SHARED, fd, (off_t)off);
    if (m == MAP_FAILED) return -1.0;
    const uint64_t samples = std::min<uint64_t>(64, npages);
    uint64_t hit = 0;
    for (uint64_t s = 0; s < samples; s++) {
        const uint64_t pg = (2 * s + 1) * npages / (2 * samples);
        unsigned char v = 0;
        if (mincore((uint8_t*)m + pg * page, page, &v) == 0) hit += v & 1;
    }
    munmap(m, len);
    return (double)hit / (double)samples;
}

}  // namespace tvi

namespace {

// The phase clock of file staging (internal counters TV_COUNTER_FILE_NS_*, tv_options_internal.h): nanoseconds a
// scope spent, added to the ctx's total for its phase (both lanes add; a lane's phases do not overlap each other).
struct FileClock {
    tv_ctx* c;
    int phase;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    FileClock(tv_ctx* ctx, int ph) : c(ctx), phase(ph) {}
    ~FileClock() {
        const auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        c->file_ns[phase].fetch_add((uint64_t)ns, std::memory_order_relaxed);
    }
};

// Memory-mapped windows of a file (the direct path), released (unregistered, unmapped) on every exit, and the open
// file.  Declared BEFORE the lane's DrainGuard, so the stream is drained before any window goes away.
struct FileWindows {
    struct W {
        void* ptr = nullptr;
        size_t len = 0;
        bool registered = false;
    };
    tv_ctx* c;
    W w[2];
    int fd = -1;
    int fd_direct = -1;           // the same file opened O_DIRECT for cold units (-2: the filesystem refused it)
    const char* path = nullptr;   // the open file (units of one segment on one lane share the open)
    uint64_t size = 0;
    explicit FileWindows(tv_ctx* ctx) : c(ctx) {}
    void release(int k) {
        if (w[k].ptr) {
            FileClock t(c, TV_FILE_PHASE_RELEASE);
            if (w[k].registered) (void)hipHostUnregister(w[k].ptr);
            munmap(w[k].ptr, w[k].len);
            (void)hipGetLastError();
        }
        w[k] = W{};
    }
    void close_file() {
        if (fd >= 0) close(fd);
        if (fd_direct >= 0) close(fd_direct);
        fd = fd_direct = -1;
        path = nullptr;
    }
    // The O_DIRECT descriptor of the open file, opened as the first one was (read + write or read-only); -1 when the
    // filesystem does not take O_DIRECT (the buffered descriptor is used then).
    void no_direct() {
        if (fd_direct >= 0) close(fd_direct);
        fd_direct = -2;
    }
    int direct_fd(bool rw) {
        if (fd_direct == -1) {
            fd_direct = open(path, (rw ? O_RDWR : O_RDONLY) | O_DIRECT | O_CLOEXEC);
            if (fd_direct < 0) fd_direct = -2;
        }
        return fd_direct >= 0 ? fd_direct : -1;
    }
    ~FileWindows() {
        release(0);
        release(1);
        close_file();
    }
};

// One part of a long file segment: file bytes [fo, fo + len) -> LINEAR [a, a + len) (inside the resident pieces),
// segment k of the call.
struct FileUnit {
    uint64_t k, fo, a, len;
    const char* path;
};

// Open the unit's file as the reference opens it (unless this lane has it open already) and check it holds the
// unit's bytes.  TV_ERR_IO (message set) when it cannot be read.
int unit_open(tv_ctx* c, FileWindows& win, const FileUnit& u) {
    FileClock t(c, TV_FILE_PHASE_OPEN);
    if (win.fd < 0 || win.path != u.path) {
        win.close_file();
        int oe = 0;
        win.fd = open_file(u.path, c->open_rw, &oe);
        if (win.fd < 0)
            return fail(c, TV_ERR_IO, "open %s for %s: %s", u.path, c->open_rw ? "read and write" : "reading",
                        strerror(oe));
        struct stat st;
        if (fstat(win.fd, &st) != 0) {
            const int e = errno;
            win.close_file();
            return fail(c, TV_ERR_IO, "fstat %s: %s", u.path, strerror(e));
        }
        win.path = u.path;
        win.size = (uint64_t)st.st_size;
    }
    if (win.size < u.fo + u.len)
        return fail(c, TV_ERR_IO, "%s has %llu bytes, the read needs %llu", u.path, (unsigned long long)win.size,
                    (unsigned long long)(u.fo + u.len));
    return TV_OK;
}

// A lane's cold-read bounce buffers: `want` of them, allocated once per context (page-locked, on the GPU's NUMA node
// when bound) and kept; each starts free.
int ensure_bounce(tv_ctx* c, int lane, int want) {
    std::lock_guard<std::mutex> g(c->bounce_mu[lane]);
    auto& v = c->bounce[lane];
    while ((int)v.size() < want) {
        Bounce b;
        TV_HIP(c, host_malloc_on_node((void**)&b.ptr, kBounceBytes, c->numa_bind ? c->numa_node : -1));
        const hipError_t e = hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
        if (e != hipSuccess) {
            (void)hipHostFree(b.ptr);
            return fail(c, TV_ERR_HIP, "hipEventCreateWithFlags: %s", hipGetErrorString(e));
        }
        v.push_back(b);
        c->bounce_free[lane].push_back((int)v.size() - 1);
    }
    return TV_OK;
}

// Cold file bytes [fo, fo + n) (O_DIRECT descriptor dfd) -> LINEAR [p, p + n) through the lane's bounce buffers
// (TV_OPT_FILE_BOUNCE = `readers`): the readers take 4 MiB parts, 4 KiB-aligned in the file, each into a free buffer
// (after the DMA that last read it), and queue the part's copies from it on the lane's stream -- the reads land in
// 2 x readers x 4 MiB of reused memory instead of across the 192 MiB ring (tools/read_ceiling.c RC_BOUNCE=dma1).
// (fo ^ p) & 3 == 0, so a part's bytes sit at the destination's alignment mod 4.  Returns a TV_ status; *read_err:
// the errno of a failed O_DIRECT read (0: none; the caller then reads the chunk again buffered).
int read_cold_bounce(tv_ctx* c, int lane, int readers, int dfd, uint64_t fo, uint64_t n, uint64_t p, int* read_err) {
    *read_err = 0;
    const uint64_t al0 = fo / 4096 * 4096, end = fo + n;
    const uint64_t nparts = (end - al0 + kBounceBytes - 1) / kBounceBytes;
    int rc = ensure_bounce(c, lane, 2 * readers);
    if (rc) return rc;
    hipStream_t cs = lane_stream(c, lane);
    std::atomic<int> err{0}, hrc{TV_OK};
    c->pool[lane].run(readers, nparts, [&](uint64_t q) {
        if (err.load(std::memory_order_relaxed) || hrc.load(std::memory_order_relaxed)) return;
        int k;
        {
            std::unique_lock<std::mutex> lk(c->bounce_mu[lane]);
            c->bounce_cv[lane].wait(lk, [&] { return !c->bounce_free[lane].empty(); });
            k = c->bounce_free[lane].back();
            c->bounce_free[lane].pop_back();
        }
        struct Give {   // the buffer goes back to the free list on every exit
            tv_ctx* c;
            int lane, k;
            ~Give() {
                {
                    std::lock_guard<std::mutex> g(c->bounce_mu[lane]);
                    c->bounce_free[lane].push_back(k);
                }
                c->bounce_cv[lane].notify_one();
            }
        } give{c, lane, k};
        Bounce& b = c->bounce[lane][k];
        if (b.recorded && hipEventSynchronize(b.ev) != hipSuccess) {
            hrc = fail(c, TV_ERR_HIP, "hipEventSynchronize of a bounce buffer failed");
            return;
        }
        const uint64_t s0 = al0 + q * kBounceBytes;                     // the file byte at b.ptr[0]
        const uint64_t a = std::max(s0, fo), e = std::min(s0 + kBounceBytes, end);
        const uint64_t want = e - s0, ask = (want + 4095) / 4096 * 4096;   // (the file's end may come back short)
        uint64_t o = 0;
        while (o < want) {
            const ssize_t got = c->file_odirect == 2 ? (errno = EINVAL, -1)   // (fault injection, as the ring path)
                                                     : pread(dfd, b.ptr + o, ask - o, (off_t)(s0 + o));
            if (got < 0 && errno == EINTR) continue;
            if (got <= 0) {
                int none = 0;
                err.compare_exchange_strong(none, got < 0 ? errno : EIO);
                return;
            }
            o += (uint64_t)got;
        }
        int r = stage_range(c, p + (a - fo), p + (e - fo), b.ptr + (a - s0), p + (a - fo), true, lane,
                            /*src_in_ring=*/true);
        if (!r && hipEventRecord(b.ev, cs) != hipSuccess) r = fail(c, TV_ERR_HIP, "hipEventRecord of a bounce buffer");
        if (r) {
            hrc = r;
            return;
        }
        b.recorded = true;
        c->file_ns[TV_FILE_BYTES_ODIRECT].fetch_add(e - a, std::memory_order_relaxed);
        c->file_ns[TV_FILE_BYTES_READ].fetch_add(e - a, std::memory_order_relaxed);
    });
    *read_err = err.load();
    return hrc.load();
}

// Stage the units (each lane's in ascending linear order) on staging lane `lane` with `threads` reader threads.
// Per chunk of the unit: with TV_OPT_FILE_DIRECT a window of TV_OPT_FILE_CHUNK bytes whose pages are mostly in the
// page cache is mapped, registered read-only and DMA'd to HBM from the page cache; otherwise (and for cold windows)
// slot-sized chunks are read by parallel preads into the lane's pinned ring and DMA'd from there.  The ring's slot
// leases order the reads behind the DMAs that last read the slot, so consecutive units stream with no drain between
// them.  A unit whose file cannot be read sets status[k] = TV_ERR_IO (the caller recovers the segment); a HIP or
// state error ends the lane with that status.
int stage_units(tv_ctx* c, const std::vector<FileUnit>& units, int lane, int threads, int32_t* status,
                bool final_pass = true) {
    if (units.empty()) return TV_OK;
    hipStream_t cs = lane_stream(c, lane);
    FileWindows win(c);  // before `drain`: unmapped after the stream is drained
    DrainGuard drain(c, lane, /*sync_compute=*/false);
    for (int k = 0; k < 2; k++) TV_HIP(c, hipEventCreateWithFlags(&drain.ev[k], hipEventDisableTiming));
    const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
    int idx = 0;
    int rc = TV_OK;
    for (const FileUnit& u : units) {
        if (unit_open(c, win, u)) {
            __atomic_store_n(&status[u.k], TV_ERR_IO, __ATOMIC_RELAXED);
            continue;
        }
        // (the pread path's chunks are one ring slot, less room for an O_DIRECT read's 4 KiB rounding)
        const uint64_t chunk = c->file_direct ? c->file_chunk : (uint64_t)kRingSlotBytes - 8192;
        bool unit_cold = false;   // the unit's bytes are mostly not in the page cache: O_DIRECT reads
        if (!c->file_direct && c->file_odirect) {
            FileClock t(c, TV_FILE_PHASE_MAP);
            const double f = cached_fraction(win.fd, u.fo, u.len);
            unit_cold = f >= 0 && f < 0.5;
        }
        bool unit_ok = true;
        for (uint64_t p = u.a; p < u.a + u.len && unit_ok; p += chunk, idx++) {
            const int k = idx & 1;
            const uint64_t n = std::min(chunk, u.a + u.len - p);
            const uint64_t fo = u.fo + (p - u.a);
            bool direct = false;
            void* m = MAP_FAILED;
            uint64_t delta = 0;
            if (c->file_direct) {
                // the window used two chunks ago must be DMA-complete before it is unmapped
                if (win.w[k].ptr) {
                    {
                        FileClock t(c, TV_FILE_PHASE_WAIT);
                        TV_HIP(c, hipEventSynchronize(drain.ev[k]));
                    }
                    win.release(k);
                }
                const uint64_t map_off = fo / page * page;
                delta = fo - map_off;
                {
                    FileClock t(c, TV_FILE_PHASE_MAP);
                    // (a file that cannot be mapped, e.g. on a filesystem without mmap, takes the pread path)
                    m = mmap(nullptr, delta + n, PROT_READ, MAP_SHARED, win.fd, (off_t)map_off);
                    if (m != MAP_FAILED) {
                        win.w[k].ptr = m;
                        win.w[k].len = delta + n;
                    }
                    // direct only when the file bytes and the resident bytes agree mod 4 (else the DMA is unaligned)
                    direct = m != MAP_FAILED && ((fo ^ p) & 3) == 0 && resident_fraction(m, delta + n, page) >= 0.5;
                }
                if (direct) {
                    // warm window: register its page-cache pages read-only and DMA them to HBM directly
                    {
                        FileClock t(c, TV_FILE_PHASE_POPULATE);
                        populate_window(m, delta + n);
                    }
                    FileClock t(c, TV_FILE_PHASE_REGISTER);
                    win.w[k].registered = hipHostRegister(m, delta + n, hipHostRegisterReadOnly) == hipSuccess;
                    (void)hipGetLastError();
                    direct = win.w[k].registered;
                }
            }
            if (direct) {
                FileClock t(c, TV_FILE_PHASE_QUEUE);
                rc = stage_range(c, p, p + n, (const uint8_t*)m + delta, p, true, lane);
                if (rc) return rc;
                c->file_ns[TV_FILE_BYTES_DIRECT].fetch_add(n, std::memory_order_relaxed);
            } else {
                // parallel preads into the pinned ring, then DMA.  A chunk whose bytes are mostly not in the page
                // cache is read with O_DIRECT (TV_OPT_FILE_ODIRECT): cold reads ran 35 % faster that way on the
                // gpurun boxes (tools/read_ceiling.c: 14.5-18.6 against 10.3-14.0 GB/s buffered, profiles/r05), and
                // the page cache keeps nothing the verify will not read again.  Its requests are whole 4 KiB blocks
                // into the slot's page-aligned start, so the chunk's bytes sit at slot + (fo % 4096): aligned for the
                // DMA when the file offset and the linear offset agree mod 4 (else the buffered read, placed at the
                // linear offset's alignment, is used).
                win.release(k);
                int dfd = (unit_cold && ((fo ^ p) & 3) == 0) ? win.direct_fd(c->open_rw) : -1;
                if (dfd >= 0 && c->file_bounce > 0) {
                    int e = 0;
                    {
                        FileClock t(c, TV_FILE_PHASE_READ);
                        rc = read_cold_bounce(c, lane, std::min(threads, c->file_bounce), dfd, fo, n, p, &e);
                    }
                    if (rc) return rc;
                    if (!e) {
                        if (c->file_direct) TV_HIP(c, hipEventRecord(drain.ev[k], cs));
                        continue;
                    }
                    // an O_DIRECT read refused: as in the ring path below, this file reads buffered from here on
                    c->file_ns[TV_FILE_ODIRECT_FALLBACKS].fetch_add(1, std::memory_order_relaxed);
                    uint64_t none = 0;
                    c->file_ns[TV_FILE_ODIRECT_ERRNO].compare_exchange_strong(none, (uint64_t)e);
                    win.no_direct();
                    dfd = -1;
                }
                const uint64_t step = dfd >= 0 ? (uint64_t)kRingSlotBytes - 8192 : (uint64_t)kRingSlotBytes - 4;
                for (uint64_t q = 0; q < n; q += step) {
                    const uint64_t kq = std::min<uint64_t>(step, n - q);
                    SlotLease slot(c, lane);  // lent until every copy out of it is queued
                    {
                        FileClock t(c, TV_FILE_PHASE_WAIT);
                        rc = slot.take();
                        if (rc) return rc;
                    }
                    uint8_t* at;
                    int e;
                    if (dfd >= 0) {
                        const uint64_t al = (fo + q) / 4096 * 4096, lead = fo + q - al;
                        at = slot.ptr() + lead;
                        FileClock t(c, TV_FILE_PHASE_READ);
                        e = c->file_odirect == 2 ? EINVAL  // (fault injection: the filesystem refusing O_DIRECT reads)
                                                 : pread_pool(c->pool[lane], threads, dfd, slot.ptr(), al,
                                                              (lead + kq + 4095) / 4096 * 4096, lead + kq);
                        if (!e) c->file_ns[TV_FILE_BYTES_ODIRECT].fetch_add(kq, std::memory_order_relaxed);
                        if (e) {
                            // an O_DIRECT read the filesystem refuses (EINVAL: alignment it does not take, a tmpfs)
                            // is not the file's failure: this file reads buffered from here on, this chunk included,
                            // and only a buffered failure counts (it is what fsStorage.get's read would see).  The
                            // fallback is counted and its first errno kept, so a systematic one (a ring slot the
                            // kernel cannot pin for direct I/O) shows (TV_FILE_ODIRECT_FALLBACKS / _ERRNO)
                            c->file_ns[TV_FILE_ODIRECT_FALLBACKS].fetch_add(1, std::memory_order_relaxed);
                            uint64_t none = 0;
                            c->file_ns[TV_FILE_ODIRECT_ERRNO].compare_exchange_strong(none, (uint64_t)e);
                            win.no_direct();
                            dfd = -1;
                            at = slot.ptr() + ((p + q) & 3);
                            e = pread_pool(c->pool[lane], threads, win.fd, at, fo + q, kq, kq);
                        }
                    } else {
                        at = slot.ptr() + ((p + q) & 3);  // at the resident bytes' alignment mod 4
                        FileClock t(c, TV_FILE_PHASE_READ);
                        e = pread_pool(c->pool[lane], threads, win.fd, at, fo + q, kq, kq);
                    }
                    if (e) {
                        fail(c, TV_ERR_IO, "read %s at %llu: %s", u.path, (unsigned long long)(fo + q), strerror(e));
                        __atomic_store_n(&status[u.k], TV_ERR_IO, __ATOMIC_RELAXED);
                        unit_ok = false;
                        break;
                    }
                    FileClock t(c, TV_FILE_PHASE_QUEUE);
                    rc = stage_range(c, p + q, p + q + kq, at, p + q, true, lane, /*src_in_ring=*/true);
                    if (rc) return rc;
                    rc = slot.release();
                    if (rc) return rc;
                    c->file_ns[TV_FILE_BYTES_READ].fetch_add(kq, std::memory_order_relaxed);
                }
            }
            if (c->file_direct) TV_HIP(c, hipEventRecord(drain.ev[k], cs));
        }
    }
    if (!final_pass && !c->file_direct) {   // (mapped page-cache windows, the direct path, must drain before unmapping)
        drain.lane_sync = false;
        return TV_OK;
    }
    FileClock t(c, TV_FILE_PHASE_DRAIN);
    TV_HIP(c, hipStreamSynchronize(cs));
    return TV_OK;
}

// tv_stage_file's work with the context lock held and the arguments checked: one segment on lane 0.
int stage_file_locked(tv_ctx* c, const char* path, uint64_t file_offset, uint64_t linear_offset, uint64_t len) {
    if (len == 0) {  // reads nothing, but fsStorage.get still opens the path (storage.ts:158)
        const int e = fs_openable(path, c->open_rw);
        return e ? fail(c, TV_ERR_IO, "open %s: %s", path, strerror(e)) : TV_OK;
    }
    FileWindows win(c);
    const FileUnit whole{0, file_offset, linear_offset, len, path};
    int rc = unit_open(c, win, whole);  // the whole segment must be readable (else TV_ERR_IO, recovered by the caller)
    win.close_file();
    if (rc || c->count == 0) return rc;
    uint64_t a, b;
    clip_to_shard(c, linear_offset, len, &a, &b);
    if (a >= b) return TV_OK;
    TV_HIP(c, hipSetDevice(c->device));
    int32_t st = TV_OK;
    rc = stage_units(c, {FileUnit{0, file_offset + (a - linear_offset), a, b - a, path}}, 0, c->file_threads, &st);
    return rc ? rc : st;
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
            __atomic_store_n(&status[sg.k], TV_ERR_IO, __ATOMIC_RELAXED);
            std::lock_guard<std::mutex> g(*err_mu);
            if (first_err->empty()) *first_err = std::string(path) + ": " + strerror(e);
        }
    });
}

// Short segments (one part each, in linear order) packed into lane `lane`'s 64 MiB ring slots at their linear
// offsets' alignment mod 4, read by the lane's pool (open, pread, close each: read_segments), one DMA per run of
// readable linear-contiguous segments while the next slot is read.  A failed read sets status[k] = TV_ERR_IO.
int stage_small(tv_ctx* c, std::vector<SmallSeg>& small, int lane, int threads, const char* const* paths,
                int32_t* status, std::string* first_err, std::mutex* err_mu, bool final_pass = true) {
    int rc = TV_OK;
    DrainGuard drain(c, lane, /*sync_compute=*/false);
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
        SlotLease slot(c, lane);  // lent until every copy out of it is queued
        {
            FileClock t(c, TV_FILE_PHASE_WAIT);
            rc = slot.take();
            if (rc) return rc;
        }
        {
            FileClock t(c, TV_FILE_PHASE_SMALL);
            read_segments(c->pool[lane], small, i, j, paths, slot.ptr(), status, threads, c->open_rw, first_err, err_mu);
        }
        FileClock t(c, TV_FILE_PHASE_QUEUE);
        for (size_t q = i; q < j;) {  // one copy per run of readable, linear-contiguous segments
            if (__atomic_load_n(&status[small[q].k], __ATOMIC_RELAXED) != TV_OK) { q++; continue; }
            size_t r = q + 1;
            while (r < j && __atomic_load_n(&status[small[r].k], __ATOMIC_RELAXED) == TV_OK &&
                   small[r].linear == small[r - 1].linear + small[r - 1].len)
                r++;
            const uint64_t lin_a = small[q].linear, lin_b = small[r - 1].linear + small[r - 1].len;
            rc = stage_range(c, lin_a, lin_b, slot.ptr() + small[q].packed, lin_a, true, lane, /*src_in_ring=*/true);
            if (rc) return rc;
            q = r;
        }
        rc = slot.release();
        if (rc) return rc;
        i = j;
    }
    if (!final_pass) {
        drain.lane_sync = false;
        return TV_OK;
    }
    FileClock t(c, TV_FILE_PHASE_DRAIN);
    TV_HIP(c, hipStreamSynchronize(lane_stream(c, lane)));
    return TV_OK;
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
    FileClock call_clock(c, TV_FILE_PHASE_CALL);
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
                     const uint64_t* linear_offsets, const uint64_t* lens, int32_t* status_out, bool check_zero,
                     bool final_pass = true) {
    int rc = TV_OK;
    // Long segments (>= TV_OPT_FILE_DIRECT_MIN bytes) are cut into units of TV_OPT_FILE_CHUNK bytes dealt to two
    // staging lanes (TV_OPT_FILE_CONCURRENT): this thread on lane 0 and a helper thread on lane 1, each walking its
    // units in linear order with its own copy stream, ring and half of the reader threads, so one file's bytes feed
    // the DMA engines from both (a whole segment per lane left a single-file torrent on one lane).  Short segments
    // are packed into lane 0's 64 MiB ring slots, read by the pool, DMA'd per run of linear-contiguous segments.
    const uint64_t direct_min = c->file_direct_min;
    std::vector<FileUnit> longs;
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
            const uint64_t unit = std::max<uint64_t>(c->file_chunk, 1ull << 20);
            for (uint64_t o = 0; o < b - a; o += unit)
                longs.push_back({k, fo + o, a + o, std::min(unit, b - a - o), paths[k]});
        } else {
            const uint64_t part = kRingSlotBytes - 4;  // (pieces of at most one slot, with room to align)
            for (uint64_t o = 0; o < b - a; o += part)
                small.push_back({k, fo + o, a + o, std::min<uint64_t>(part, b - a - o), 0});
            small_bytes += b - a;
        }
    }
    // Short segments: with two lanes, the first half (by bytes, in linear order) on lane 0 and the second on lane 1
    // once there are at least two slots of them, so one lane's reads overlap the other's DMA and wait (each lane reads
    // a slot, queues its DMA, and waits for a free slot in turn)
    // (a context with one host thread stages on one lane: a second lane would be a second thread)
    const bool concurrent = c->file_concurrent && c->file_threads >= 2;
    std::vector<SmallSeg> lane_small[2];
    {
        std::stable_sort(small.begin(), small.end(), [](const SmallSeg& x, const SmallSeg& y) { return x.linear < y.linear; });
        const bool split = concurrent && small_bytes >= 2 * (uint64_t)kRingSlotBytes;
        uint64_t acc = 0;
        for (const SmallSeg& sg : small) {
            lane_small[split && acc >= small_bytes / 2 ? 1 : 0].push_back(sg);
            acc += sg.len;
        }
    }
    uint64_t small_load[2] = {0, 0};
    for (int l = 0; l < 2; l++)
        for (const SmallSeg& sg : lane_small[l]) small_load[l] += sg.len;
    // in linear order, each unit to the lane with fewer bytes so far
    std::vector<FileUnit> lane_units[2];
    {
        std::stable_sort(longs.begin(), longs.end(), [](const FileUnit& x, const FileUnit& y) { return x.a < y.a; });
        uint64_t load[2] = {small_load[0], small_load[1]};
        for (const FileUnit& u : longs) {
            const int l = (concurrent && load[1] < load[0]) ? 1 : 0;
            lane_units[l].push_back(u);
            load[l] += u.len;
        }
    }
    // reader threads: the context's TV_OPT_FILE_THREADS shared by the lanes that read
    const int lanes = (lane_units[1].empty() && lane_small[1].empty()) ? 1 : 2;
    const int threads_per_lane = std::max(1, c->file_threads / lanes);
    // (everything the helper touches is declared before the joiner, so an early return joins it first)
    std::string first_err = zero_err;
    std::mutex err_mu;
    int helper_rc = TV_OK;
    std::thread helper;
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{helper};  // every exit joins the helper before the ctx lock is released
    if (lanes == 2) {
        helper = std::thread([&]() {
            pin_thread(numa_cpus(c));  // next to its ring and the GPU (TV_OPT_NUMA_BIND)
            if (hipSetDevice(c->device) != hipSuccess) {
                helper_rc = fail(c, TV_ERR_HIP, "tv_stage_files: hipSetDevice(%d) failed", c->device);
                return;
            }
            helper_rc = stage_units(c, lane_units[1], 1, threads_per_lane, status_out, final_pass);
            if (!helper_rc && !lane_small[1].empty())
                helper_rc = stage_small(c, lane_small[1], 1, threads_per_lane, paths, status_out, &first_err, &err_mu,
                                        final_pass);
        });
    }
    rc = stage_units(c, lane_units[0], 0, lanes == 2 ? threads_per_lane : c->file_threads, status_out, final_pass);
    if (rc) return rc;
    if (!lane_small[0].empty()) {
        rc = stage_small(c, lane_small[0], 0, lanes == 2 ? threads_per_lane : c->file_threads, paths, status_out,
                         &first_err, &err_mu, final_pass);
        if (rc) return rc;
    }
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

int stage_files_locked(tv_ctx* c, uint64_t n, const char* const* paths, const uint64_t* file_offsets,
                       const uint64_t* linear_offsets, const uint64_t* lens, int32_t* status_out);

}  // namespace

extern "C" {

int tv_stage_files(tv_ctx* c, uint64_t n, const char* const* paths, const uint64_t* file_offsets,
                   const uint64_t* linear_offsets, const uint64_t* lens, int32_t* status_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    FileClock call_clock(c, TV_FILE_PHASE_CALL);
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
    return stage_files_locked(c, n, paths, file_offsets, linear_offsets, lens, status_out);
}

int tv_stage_file_table(tv_ctx* c, uint64_t n, const uint64_t* lengths, const char* paths, uint64_t paths_bytes,
                        int32_t* status_out) {
    if (!c) return fail(nullptr, TV_ERR_ARG, "ctx is NULL");
    std::lock_guard<std::mutex> g(c->mu);
    FileClock call_clock(c, TV_FILE_PHASE_CALL);
    int rc = require_layout(c, false, true);
    if (rc) return rc;
    if (n == 0) return TV_OK;
    if (!lengths || !paths || !status_out) return fail(c, TV_ERR_ARG, "NULL argument");
    // file k's path: the k-th NUL-terminated string of the buffer
    std::vector<const char*> path(n);
    uint64_t o = 0;
    for (uint64_t k = 0; k < n; k++) {
        const void* z = o < paths_bytes ? memchr(paths + o, 0, paths_bytes - o) : nullptr;
        if (!z)
            return fail(c, TV_ERR_ARG, "paths holds %llu NUL-terminated paths in %llu bytes, the table %llu files",
                        (unsigned long long)k, (unsigned long long)paths_bytes, (unsigned long long)n);
        path[k] = paths + o;
        o = (uint64_t)((const char*)z - paths) + 1;
        status_out[k] = TV_OK;
    }
    if (c->count == 0) return TV_OK;
    // findAndDo's walk over the files in order (storage.ts:98-137), restricted to the shard's bytes (tv_plan.h)
    const uint64_t last = c->first + c->count - 1;
    const uint64_t lo = c->first * c->L, hi = std::min(c->total, last * c->L + piece_len(c, last));
    std::vector<TableSeg> segs;
    uint64_t bad = 0, reached = 0;
    if (!walk_file_table(n, lengths, lo, hi, c->L, &segs, &bad, &reached))
        return fail(c, TV_ERR_ARG, "file %llu: the lengths overflow 64-bit offsets", (unsigned long long)bad);
    std::vector<const char*> sp;
    std::vector<uint64_t> sfo, slin, slen;
    for (const TableSeg& g : segs) {
        sp.push_back(path[g.file]);
        sfo.push_back(g.file_offset);
        slin.push_back(g.linear);
        slen.push_back(g.len);
    }
    std::vector<int32_t> st(sp.size(), TV_OK);
    if (!sp.empty()) rc = stage_files_locked(c, sp.size(), sp.data(), sfo.data(), slin.data(), slen.data(), st.data());
    for (size_t q = 0; q < sp.size(); q++)
        if (st[q] != TV_OK) status_out[segs[q].file] = st[q];
    // the files end before the shard does: Storage.get's walk for a piece past their end never completes (null)
    if (!rc && reached < hi) mark_bad(c, reached, hi);
    return rc;
}

}  // extern "C"

namespace {

// tv_stage_files' work with the lock held and the segments checked (status_out preset to TV_OK).
int stage_files_locked(tv_ctx* c, uint64_t n, const char* const* paths, const uint64_t* file_offsets,
                       const uint64_t* linear_offsets, const uint64_t* lens, int32_t* status_out) {
    int rc = TV_OK;
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
    uint64_t last_touched = 0;
    for (uint64_t w = 0; w < nwin; w++)
        if (touched[w]) last_touched = w;
    for (uint64_t w = 0; w < nwin; w++) {
        if (!touched[w]) continue;
        rc = win_enter(c, w);
        // (the lanes flow from one window's pass into the next; only the last pass drains them)
        if (!rc) rc = stage_files_core(c, n, paths, file_offsets, linear_offsets, lens, status_out, check_zero,
                                       w == last_touched);
        if (rc) {
            (void)hipStreamSynchronize(c->copy_stream);
            (void)hipStreamSynchronize(c->copy_stream2);
            return rc;
        }
        check_zero = false;
    }
    return check_zero ? stage_files_core(c, n, paths, file_offsets, linear_offsets, lens, status_out, true) : TV_OK;
}

}  // namespace
