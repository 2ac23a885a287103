// tv_api.hip -- C ABI of libtorrent_verify.so (declared in include/torrent_verify.h).
//
// Owns, per context (= per GPU): the compute stream, two staging lanes (a copy stream and a ring of
// pinned host staging buffers each), timing events, and the device allocations (resident payload
// with padded piece stride, digests, availability / output bitfields, chaining state for streamed
// runs).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/torrent_verify.h"
#include "tv_host.h"
#include "tv_internal.h"

namespace {

thread_local std::string g_thread_error;

constexpr uint64_t kSlack = 256;                          // bytes past the last resident piece (tail over-read)
constexpr int kRingSlots = TV_STREAM_RING_SLOTS;          // pinned staging buffers per lane
constexpr size_t kRingSlotBytes = TV_STREAM_SLOT_BYTES;

// Pin the calling thread to `cpus` (nullptr: leave it).  Used for the library's own threads only.
void pin_thread(const cpu_set_t* cpus) {
    if (cpus) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), cpus);
}

// The NUMA node of GPU `device` (its PCI function's numa_node in sysfs), or -1.
int gpu_numa_node(int device) {
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, (int)sizeof bdf, device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char* p = bdf; *p; p++) *p = (char)tolower((unsigned char)*p);
    const std::string path = std::string("/sys/bus/pci/devices/") + bdf + "/numa_node";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    return node;
}

// The CPUs of NUMA node `node` that this process may run on (sysfs cpulist & sched_getaffinity).
bool node_cpus(int node, cpu_set_t* out) {
    CPU_ZERO(out);
    if (node < 0) return false;
    char path[96];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE* f = fopen(path, "r");
    if (!f) return false;
    char list[4096] = {0};
    const bool got = fgets(list, sizeof list, f) != nullptr;
    fclose(f);
    if (!got) return false;
    for (char* p = list; *p && *p != '\n';) {
        char* end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p) break;
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            p = end;
        }
        for (long cpu = a; cpu <= b && cpu < CPU_SETSIZE; cpu++) CPU_SET((int)cpu, out);
        if (*p == ',') p++;
    }
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0) CPU_AND(out, out, &allowed);
    return CPU_COUNT(out) > 0;
}

// hipHostMalloc with the pages placed on NUMA node `node` (>= 0): the calling thread's memory policy is set
// to prefer that node around the allocation (hipHostMallocNumaUser makes HIP follow it) and restored.
hipError_t host_malloc_on_node(void** p, size_t bytes, int node) {
    if (node < 0 || node >= 1024) return hipHostMalloc(p, bytes, hipHostMallocDefault);
    int old_mode = 0;
    unsigned long old_mask[16] = {0};
    if (syscall(SYS_get_mempolicy, &old_mode, old_mask, 1024ul, nullptr, 0ul) != 0)
        return hipHostMalloc(p, bytes, hipHostMallocDefault);
    unsigned long mask[16] = {0};
    mask[node / 64] = 1ul << (node % 64);
    constexpr int kMpolPreferred = 1;
    if (syscall(SYS_set_mempolicy, kMpolPreferred, mask, 1024ul) != 0)
        return hipHostMalloc(p, bytes, hipHostMallocDefault);
    hipError_t e = hipHostMalloc(p, bytes, hipHostMallocNumaUser);
    (void)syscall(SYS_set_mempolicy, old_mode, old_mode ? old_mask : nullptr, old_mode ? 1024ul : 0ul);
    if (e != hipSuccess) {  // a runtime without the flag: default placement
        (void)hipGetLastError();
        e = hipHostMalloc(p, bytes, hipHostMallocDefault);
    }
    return e;
}

// The NUMA node holding the page at `p` (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), or -1.
int page_node(const void* p) {
    int node = -1;
    constexpr unsigned long kFNode = 1, kFAddr = 2;
    if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0ul, p, kFNode | kFAddr) != 0) return -1;
    return node;
}

// Persistent host workers (one pool per staging lane): run(threads, tasks, fn) calls fn(0..tasks-1) on up
// to `threads` threads, the caller included, and returns when every task is done.  Spawning threads for
// every 64 MiB staging slot cost ~0.3 ms a slot, a quarter of the slot's PCIe time.  With an affinity set
// (the GPU's NUMA node, TV_OPT_NUMA_BIND) the workers run on those CPUs and the caller only waits, so every
// copy into the pinned ring runs next to the ring's memory and the GPU.
class Pool {
  public:
    // cpus: where the workers run (nullptr: unpinned, i.e. on `process`, the process's CPUs recorded once at
    // tv_create -- not a worker's own mask, which a thread inherits from its creator: lane 1's workers are
    // created by the staging helper thread, itself pinned to the GPU's node)
    void set_affinity(const cpu_set_t* cpus, const cpu_set_t* process) {
        std::lock_guard<std::mutex> g(mu_);
        has_aff_ = cpus != nullptr;
        if (cpus) aff_ = *cpus;
        has_all_ = process != nullptr;
        if (process) all_ = *process;
        aff_gen_++;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(int threads, uint64_t tasks, const std::function<void(uint64_t)>& fn) {
        const uint64_t t = std::min<uint64_t>((uint64_t)std::max(1, threads), tasks);
        if (t <= 1) {
            for (uint64_t q = 0; q < tasks; q++) fn(q);
            return;
        }
        std::unique_lock<std::mutex> lk(mu_);
        const bool caller_works = !has_aff_;
        const uint64_t workers = caller_works ? t - 1 : t;
        while (th_.size() < workers) th_.emplace_back([this] { loop(); });
        fn_ = &fn;
        tasks_ = tasks;
        next_ = 0;
        open_ = (int)workers;
        gen_++;
        lk.unlock();
        cv_.notify_all();
        if (caller_works) work();
        lk.lock();
        done_.wait(lk, [&] { return next_ >= tasks_; });  // (unpinned caller: every task claimed)
        open_ = 0;  // no late joiner may start on this run once the caller has seen every task claimed
        done_.wait(lk, [&] { return running_ == 0; });
    }

  private:
    void work() {
        for (uint64_t q = next_++; q < tasks_; q = next_++) (*fn_)(q);
    }
    void loop() {
        uint64_t seen = 0, aff_seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || (gen_ != seen && open_ > 0); });
            if (stop_) return;
            seen = gen_;
            open_--;
            running_++;
            if (aff_seen != aff_gen_) {
                aff_seen = aff_gen_;
                if (has_aff_) pin_thread(&aff_);
                else if (has_all_) pin_thread(&all_);
            }
            lk.unlock();
            work();
            lk.lock();
            if (--running_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(uint64_t)>* fn_ = nullptr;
    uint64_t tasks_ = 0;
    std::atomic<uint64_t> next_{0};
    int open_ = 0, running_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    bool has_aff_ = false, has_all_ = false;
    cpu_set_t aff_, all_;
    uint64_t aff_gen_ = 0;
};

// One streamed verify (tv_stream_*): units of C bytes of every piece of a window of shard pieces flow host ->
// pinned ring slot -> device chunk buffer (two, ping-pong) -> one kernel launch per unit.  Column mode: one
// window (the shard), C-byte columns.  Row mode (TV_OPT_STREAM_ROWS): C = the whole piece, windows of wn pieces.
struct StreamState {
    bool active = false;
    bool outstanding = false;  // a request (and its ring slot) is lent to the caller
    int slot = -1;             // the lent ring slot (lane 0)
    tv_stream_req req{};
    uint64_t C = 0, row_pitch = 0, ncol = 0, row = 0, rows_per_req = 0, seq = 0;
    uint64_t wn = 0, nwin = 0, unit = 0, nunits = 0;  // pieces per window, windows; unit = window * ncol + column
    int kernel = 0;
    bool k0 = false;           // ev_k0 recorded (first launch queued)
    std::vector<uint8_t> av;   // shard-relative availability bits, applied to the bitfield at the end
};

}  // namespace

struct tv_ctx {
    int device = 0;
    std::mutex mu;
    std::string err;

    hipStream_t stream = nullptr;       // kernels
    hipStream_t copy_stream = nullptr;  // H2D staging
    hipStream_t copy_stream2 = nullptr; // H2D staging of the second lane (tv_stage_files' long segments)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;  // TV_OPT_TWIN_PACK launches on pack_stream
    int cus = 256;                      // compute units of the device
    hipEvent_t ev_call0 = nullptr, ev_k0 = nullptr, ev_k1 = nullptr, ev_call1 = nullptr;

    // geometry
    bool has_layout = false;
    uint64_t total = 0, L = 0, P = 0, first = 0, count = 0;
    uint64_t stride = 0;
    // options
    int kernel_opt = TV_KERNEL_AUTO;
    uint64_t pad = 256;
    uint64_t stream_chunk = 0;  // 0 = automatic
    int split_pairs = 0;        // 0 = automatic
    uint64_t file_chunk = 256ull << 20;  // tv_stage_file: bytes per mapped window
    bool file_direct = true;             // tv_stage_file: DMA from registered page-cache pages
    bool file_concurrent = true;         // tv_stage_files: long segments on two staging lanes
    uint64_t file_direct_min = 32ull << 20;  // tv_stage_files: segments >= this take the tv_stage_file path
    int file_threads = 16;                   // tv_stage_files: reader threads
    bool resident = true;                    // TV_OPT_RESIDENT
    bool debug_rebounce = false;             // TV_OPT_DEBUG_REBOUNCE
    bool twin_pack = false;                  // TV_OPT_TWIN_PACK
    int twin_fill = 1;                       // TV_OPT_TWIN_FILL: 0 off, 1 auto, 2 also on short lists
    bool fill_all = false;                   // TV_OPT_TWIN_FILL_READS
    hipStream_t pack_stream = nullptr;       // twin launches CU-masked to pack_cus CUs (TV_OPT_TWIN_PACK)
    int pack_cus = 0;

    // allocation capacities (tv_set_layout reuses what fits)
    uint64_t cap_payload = 0;   // bytes of d_payload
    uint64_t cap_count = 0;     // pieces of d_digests / d_state / d_hash
    uint64_t cap_words = 0;     // 64-bit words of d_avail / d_base_avail / h_avail / d_out

    // device memory
    uint8_t* d_payload = nullptr;
    uint32_t* d_digests = nullptr;    // [5][count]
    uint64_t* d_avail = nullptr;      // bit words, sized to whole 256-piece groups (caller-masked)
    uint64_t* d_base_avail = nullptr; // same shape: digest slice complete & piece inside the torrent
    uint8_t* h_avail = nullptr;       // pinned bounce buffer for caller-masked availability
    hipEvent_t ev_avail = nullptr;    // the last H2D copy out of h_avail
    uint64_t* d_out = nullptr;
    uint32_t* d_state = nullptr;      // [5][count]
    uint32_t* d_hash = nullptr;       // [5][count]
    uint8_t* d_chunk[2] = {nullptr, nullptr};
    uint32_t* d_list = nullptr;       // tv_verify_list indices
    uint8_t* d_list_out = nullptr;
    uint64_t list_cap = 0;
    uint64_t chunk_bytes = 0;
    size_t bit_words = 0;

    bool digests_set = false;
    std::vector<uint8_t> digest_ok;   // shard-relative MSB-first bits: digest slice is 20 bytes
    std::vector<uint8_t> base_avail;  // host copy of d_base_avail (bit_words * 8 bytes)
    // shard-relative MSB-first bits of the pieces a tv_stage_file(s) call could not read as fsStorage.get
    // reads them (until the next tv_set_layout); tv_verify reports them 0
    std::vector<uint8_t> file_bad;
    bool any_file_bad = false;

    // pinned staging ring.  A slot is LENT from take_slot until release_slot records its event after the
    // last copy queued from it; take_slot never hands out a lent slot (it takes the next free one), so a
    // copy can never be overwritten by a later take of the same lane, whatever the DMA timing.
    uint8_t* ring[kRingSlots] = {nullptr, nullptr, nullptr};
    hipEvent_t ring_ev[kRingSlots] = {nullptr, nullptr, nullptr};
    bool ring_lent[kRingSlots] = {false, false, false};
    int ring_next = 0;
    // lane 1 (copy_stream2 + ring2): tv_stage_files runs its long segments on it beside the reader pool
    uint8_t* ring2[kRingSlots] = {nullptr, nullptr, nullptr};
    hipEvent_t ring2_ev[kRingSlots] = {nullptr, nullptr, nullptr};
    bool ring2_lent[kRingSlots] = {false, false, false};
    int ring2_next = 0;
    Pool pool[2];                     // host workers of lane 0 / lane 1
    // the GPU's NUMA node (-1: unknown) and its CPUs the process may use; with numa_bind the library's
    // threads run there and the pinned ring is allocated there (TV_OPT_NUMA_BIND)
    int numa_node = -1;
    bool numa_cpus_ok = false;
    cpu_set_t numa_cpus;
    bool numa_bind = true;
    std::mutex err_mu;                // fail() may run on a tv_stage_files helper thread
    uint8_t* h_bits = nullptr;        // pinned bitfield bounce buffer
    size_t h_bits_cap = 0;

    // streamed verify (tv_stream_*)
    StreamState st;
    hipEvent_t col_ev[2] = {nullptr, nullptr};   // copies of the column into chunk buffer k queued before it
    hipEvent_t done_ev[2] = {nullptr, nullptr};  // the kernel that last read chunk buffer k

    // counters (tv_get_counter): device allocations since tv_create
    uint64_t n_payload_allocs = 0, n_device_allocs = 0;

    // last call
    float kernel_ms = 0.f, total_ms = 0.f;
    int last_kernel = 0, last_launches = 0;
    uint32_t last_workgroups = 0;      // grid of the last verify / hash / list launch, companions included

    // Device budget (TV_OPT_RESIDENT_BUDGET).  A shard whose padded payload exceeds it gets a WINDOWED layout:
    // the payload allocation holds win_bufs buffers of win_n pieces, each window is hashed (HASH kernels into
    // d_hash) as soon as staging moves past it, while the next window stages into the other buffer, and
    // tv_verify compares d_hash with the digests at the end.  Staging must then ascend window by window.
    uint64_t budget_opt = 0;           // bytes; 0 = automatic (free HBM at tv_set_layout - a margin)
    uint64_t budget = 0;               // the budget the last tv_set_layout applied (0: no resident payload)
    bool win = false;                  // the layout is windowed
    uint64_t win_n = 0;                // pieces per window
    int win_bufs = 0;                  // buffers in d_payload (2: window k + 1 stages while k hashes; 1)
    uint64_t win_buf_bytes = 0;        // bytes per buffer (win_n * stride + kSlack)
    uint64_t win_cur = UINT64_MAX;     // window open for staging (UINT64_MAX: none)
    int win_buf = 1;                   // its buffer
    uint64_t win_valid = 0;            // shard pieces [0, win_valid) are hashed (or zeroed: never staged) this pass
    bool win_done = false;             // the pass is finalized: d_hash holds every shard piece's digest
    bool win_timing = false;           // ev_call0 / ev_k0 recorded for this pass
    uint64_t win_launched = 0;         // windows hashed this pass
    uint64_t win_passes = 0;           // passes finalized since tv_set_layout
    hipEvent_t win_ev[2] = {nullptr, nullptr};  // the last kernel reading buffer k
    hipEvent_t win_cp[2] = {nullptr, nullptr};  // copies into the window queued on lane k (kernel waits on them)

    // Slot pool (TV_OPT_LIST_SLOTS = K): the payload holds K piece slots instead of the shard; a staged piece
    // takes a slot until tv_verify_list lists it (incremental verify).
    uint64_t list_slots_opt = 0;
    uint64_t slots = 0;                // slots of the current layout (0: not a slot layout)
    std::unordered_map<uint64_t, uint32_t> slot_of;  // shard-relative piece -> slot
    std::vector<uint32_t> slot_free;

    bool open_rw = true;               // TV_OPT_OPEN_RW: files opened read + write (fsStorage.get) or read-only
    bool stream_rows = false;          // TV_OPT_STREAM_ROWS: stream requests carry whole pieces (windows of pieces)
    int lane_pairs = 0;                // TV_OPT_LANE_PAIRS: 0 auto (>= 256 x CUs pieces in the launch), 1 on, 2 off
    bool clock_probe = false;          // TV_OPT_CLOCK_PROBE: verify / hash launches stamp their clock into d_clock
    uint64_t* d_clock = nullptr;       // {shader clock, real-time} counters at the start and end of workgroup 0
    cpu_set_t proc_cpus;               // the process's CPUs at tv_create (what "unpinned" workers run on)
    bool proc_cpus_ok = false;
};

namespace {

int fail(tv_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) {
        std::lock_guard<std::mutex> g(c->err_mu);
        c->err = buf;
    }
    g_thread_error = buf;
    return code;
}

#define TV_HIP(c, call)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail((c), e_ == hipErrorOutOfMemory ? TV_ERR_NOMEM : TV_ERR_HIP, "%s: %s (%s:%d)", #call, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                             \
    } while (0)

uint64_t piece_len(const tv_ctx* c, uint64_t i) {  // piece.ts:16-19
    if (i == c->P - 1 && c->total % c->L) return c->total % c->L;
    return c->L;
}

inline void set_bit(uint8_t* bf, uint64_t i) { bf[i >> 3] |= (uint8_t)(0x80u >> (i & 7)); }
inline bool get_bit(const uint8_t* bf, uint64_t i) { return (bf[i >> 3] >> (7 - (i & 7))) & 1; }

// May this process open the existing file `path` as the caller's reference path opens it?  rw (TV_OPT_OPEN_RW,
// the default): read + write, as fsStorage.get opens every segment ({read, write, create}, storage.ts:28-32,158);
// else read-only, as make_torrent.ts:78 opens its sources (Deno.open's default).  0, or the errno.
int access_ok(const char* path, bool rw) {
    return faccessat(AT_FDCWD, path, rw ? (R_OK | W_OK) : R_OK, AT_EACCESS) == 0 ? 0 : errno;
}


// Open an existing file for reading the way the reference opens it: read + write for fsStorage.get
// (storage.ts:28-32,158; -1 where that open fails: no write permission, a directory, a read-only filesystem),
// read-only for make_torrent.ts:78 (creation from files the process may not write).  One open walks the path
// once; an access(R_OK | W_OK) check before an O_RDONLY open walked it twice and was 4-5 % slower on 10,000
// small files (profiles/r03/f2_numa_ab.jsonl).  Nothing is ever written.
int open_file(const char* path, bool rw, int* err) {
    const int fd = open(path, (rw ? O_RDWR : O_RDONLY) | O_CLOEXEC);
    *err = fd < 0 ? errno : 0;
    return fd;
}

// Would fsStorage.get's Deno.open(path, {read, write, create}) succeed (storage.ts:28-32,158)?  Checked
// without creating anything: an existing non-directory this process may read and write, or a missing file
// whose parent directory exists and may be written.  A zero-length segment of Storage.get's walk
// (storage.ts:109-110: a file ending where the piece starts, or a zero-length file inside the piece) reads
// nothing, but its open still decides whether the piece is null.  Read-only mode (!rw, make_torrent.ts:78's
// Deno.open(path)): an existing readable non-directory; a missing file fails (nothing would create it).
// 0, or the errno.
int fs_openable(const char* path, bool rw) {
    if (!path[0]) return ENOENT;
    struct stat st;
    if (stat(path, &st) == 0) return S_ISDIR(st.st_mode) ? EISDIR : access_ok(path, rw);
    if (errno != ENOENT || !rw) return errno;
    std::string parent(path);
    const size_t cut = parent.find_last_of('/');
    parent = cut == std::string::npos ? std::string(".") : (cut == 0 ? std::string("/") : parent.substr(0, cut));
    if (stat(parent.c_str(), &st) != 0) return errno;          // a missing parent directory: open fails
    if (!S_ISDIR(st.st_mode)) return ENOTDIR;
    return faccessat(AT_FDCWD, parent.c_str(), W_OK | X_OK, AT_EACCESS) == 0 ? 0 : errno;
}

void free_payload(tv_ctx* c) {
    (void)hipFree(c->d_payload); c->d_payload = nullptr;
    c->cap_payload = 0;
}

void free_per_piece(tv_ctx* c) {
    (void)hipFree(c->d_digests); c->d_digests = nullptr;
    (void)hipFree(c->d_state); c->d_state = nullptr;
    (void)hipFree(c->d_hash); c->d_hash = nullptr;
    c->cap_count = 0;
}

void free_words(tv_ctx* c) {
    (void)hipFree(c->d_avail); c->d_avail = nullptr;
    (void)hipFree(c->d_base_avail); c->d_base_avail = nullptr;
    if (c->ev_avail) (void)hipEventSynchronize(c->ev_avail);
    (void)hipHostFree(c->h_avail); c->h_avail = nullptr;
    (void)hipFree(c->d_out); c->d_out = nullptr;
    c->cap_words = 0;
}

void free_chunks(tv_ctx* c) {
    for (auto& p : c->d_chunk) { (void)hipFree(p); p = nullptr; }
    c->chunk_bytes = 0;
}

void free_list(tv_ctx* c) {
    (void)hipFree(c->d_list); c->d_list = nullptr;
    (void)hipFree(c->d_list_out); c->d_list_out = nullptr;
    c->list_cap = 0;
}

void free_device(tv_ctx* c) {
    free_payload(c);
    free_per_piece(c);
    free_words(c);
    free_chunks(c);
    free_list(c);
}

// An allocation of `cap` units is reused for `need` units when it holds them and is not more than twice
// (or 64 Mi units) larger: a stream of small layouts after a big one must not pin the big one forever.
bool reuse_fits(uint64_t need, uint64_t cap) {
    return need <= cap && (cap <= (64ull << 20) || need >= cap / 2);
}

// Staging lane `which`: 0 = copy_stream + ring, 1 = copy_stream2 + ring2.  Lane 1 is used only by
// tv_stage_files' helper thread, so the two lanes never share a ring slot or a stream.
struct RingRef {
    uint8_t** buf;
    hipEvent_t* ev;
    bool* lent;
    int* next;
};
RingRef ring_ref(tv_ctx* c, int which) {
    return which ? RingRef{c->ring2, c->ring2_ev, c->ring2_lent, &c->ring2_next}
                 : RingRef{c->ring, c->ring_ev, c->ring_lent, &c->ring_next};
}

hipStream_t lane_stream(const tv_ctx* c, int which) { return which ? c->copy_stream2 : c->copy_stream; }

// The CPUs the context's library threads run on: the GPU's NUMA node when bound, else none (unpinned).
const cpu_set_t* numa_cpus(const tv_ctx* c) { return (c->numa_bind && c->numa_cpus_ok) ? &c->numa_cpus : nullptr; }

void apply_numa(tv_ctx* c) {
    for (auto& p : c->pool) p.set_affinity(numa_cpus(c), c->proc_cpus_ok ? &c->proc_cpus : nullptr);
}

int ensure_ring(tv_ctx* c, int which = 0) {
    RingRef r = ring_ref(c, which);
    for (int s = 0; s < kRingSlots; s++) {
        if (!r.buf[s])
            TV_HIP(c, host_malloc_on_node((void**)&r.buf[s], kRingSlotBytes, c->numa_bind ? c->numa_node : -1));
        if (!r.ev[s]) TV_HIP(c, hipEventCreateWithFlags(&r.ev[s], hipEventDisableTiming));
    }
    return TV_OK;
}

int ensure_hbits(tv_ctx* c, size_t bytes) {
    if (c->h_bits_cap >= bytes) return TV_OK;
    if (c->h_bits) (void)hipHostFree(c->h_bits);
    c->h_bits = nullptr;
    c->h_bits_cap = 0;
    TV_HIP(c, hipHostMalloc((void**)&c->h_bits, bytes, hipHostMallocDefault));
    c->h_bits_cap = bytes;
    return TV_OK;
}

// Lend the next free pinned ring slot of lane `which` (waiting for the copies queued from it before its
// last release).  A slot that is still lent -- the source of copies that are being queued right now -- is
// never handed out: the next free one is taken instead.  All lent: TV_ERR_STATE (a caller bug, never a
// silent overwrite).
int take_slot(tv_ctx* c, int* slot, int which = 0) {
    int rc = ensure_ring(c, which);
    if (rc) return rc;
    RingRef r = ring_ref(c, which);
    for (int k = 0; k < kRingSlots; k++) {
        const int s = (*r.next + k) % kRingSlots;
        if (r.lent[s]) continue;
        *r.next = (s + 1) % kRingSlots;
        TV_HIP(c, hipEventSynchronize(r.ev[s]));
        r.lent[s] = true;
        *slot = s;
        return TV_OK;
    }
    return fail(c, TV_ERR_STATE, "every staging slot of lane %d is lent out", which);
}

// Return a lent slot: its event is recorded on the lane's copy stream, after every copy queued from it.
int release_slot(tv_ctx* c, int slot, int which = 0) {
    RingRef r = ring_ref(c, which);
    r.lent[slot] = false;
    TV_HIP(c, hipEventRecord(r.ev[slot], lane_stream(c, which)));
    return TV_OK;
}

// A lent slot that goes back to the ring on every exit of its scope (error paths included).
struct SlotLease {
    tv_ctx* c;
    int lane;
    int s = -1;
    SlotLease(tv_ctx* ctx, int l) : c(ctx), lane(l) {}
    ~SlotLease() {
        if (s >= 0) (void)release_slot(c, s, lane);
        (void)hipGetLastError();
    }
    SlotLease(const SlotLease&) = delete;
    SlotLease& operator=(const SlotLease&) = delete;
    int take() { return take_slot(c, &s, lane); }
    int release() {
        const int k = s;
        s = -1;
        return k >= 0 ? release_slot(c, k, lane) : TV_OK;
    }
    uint8_t* ptr() const { return ring_ref(c, lane).buf[s]; }
};

// Base availability of every shard piece, computed once per tv_set_digests and kept in HBM: the
// digest slice is complete (metainfo.ts:111) and the piece's bytes lie inside the torrent (piece.ts:16-19
// length at offset i*L must end <= total).
int upload_base_avail(tv_ctx* c) {
    const size_t nbytes = c->bit_words * 8;
    std::vector<uint8_t> bits(nbytes, 0);
    for (uint64_t j = 0; j < c->count; j++) {
        const uint64_t i = c->first + j;
        if (get_bit(c->digest_ok.data(), j) && i * c->L + piece_len(c, i) <= c->total) set_bit(bits.data(), j);
    }
    TV_HIP(c, hipMemcpyAsync(c->d_base_avail, bits.data(), nbytes, hipMemcpyHostToDevice, c->stream));
    TV_HIP(c, hipStreamSynchronize(c->stream));
    c->base_avail.swap(bits);
    return TV_OK;
}

// Availability for one launch: the base bits, or base & the caller's bits (Storage.get -> null for
// a missing / short file) & not the pieces file staging could not read, queued on the compute stream from
// the pinned bounce buffer (no host sync).
int launch_avail(tv_ctx* c, const uint8_t* avail_bits, const uint64_t** out) {
    if (!avail_bits && !c->any_file_bad) {
        *out = c->d_base_avail;
        return TV_OK;
    }
    TV_HIP(c, hipEventSynchronize(c->ev_avail));  // the previous copy out of h_avail is done
    const size_t nbytes = c->bit_words * 8, used = (c->count + 7) / 8;
    for (size_t k = 0; k < nbytes; k++) {
        const uint8_t caller = k < used ? (avail_bits ? avail_bits[k] : 0xFF) : 0;
        const uint8_t bad = k < used ? c->file_bad[k] : 0;
        c->h_avail[k] = c->base_avail[k] & caller & (uint8_t)~bad;
    }
    TV_HIP(c, hipMemcpyAsync(c->d_avail, c->h_avail, nbytes, hipMemcpyHostToDevice, c->stream));
    TV_HIP(c, hipEventRecord(c->ev_avail, c->stream));
    *out = c->d_avail;
    return TV_OK;
}

// Kernel of a launch over n consecutive pieces, one of them the torrent's short last piece when short_last
// (resident calls, windows of a windowed layout and streamed columns alike).
int choose_kernel_n(const tv_ctx* c, uint64_t n, bool short_last) {
    if (c->kernel_opt == TV_KERNEL_LANE || c->kernel_opt == TV_KERNEL_SPLIT || c->kernel_opt == TV_KERNEL_TWIN)
        return c->kernel_opt;
    // Twin (two lanes per piece, 2-wave workgroups over 32 pieces, 60 KiB of LDS: two per CU) while every
    // wave has a SIMD to itself: <= 2 workgroups per CU, i.e. 16,384 pieces on 256 CUs (cfg2 1,419 vs split
    // 1,326 GB/s; +5-6 % at 4,096-12,800 pieces, profiles/r02/sweep_twin.log).  Then split (schedule offload)
    // while every split pair (64 pieces, 2 waves) has SIMDs to itself: <= 32,768 pieces.  Beyond that rounds
    // waves share SIMDs and the lane kernel wins (measured 40,960 pieces split 1.62 vs lane 2.33 TB/s; 32,768
    // split 2.50 vs lane 1.87).
    const uint64_t n_main = n - (short_last ? 1 : 0);
    const uint64_t twin_wgs = (n_main + 31) / 32 + (short_last ? 1 : 0);   // as tv_launch_verify
    if (c->split_pairs != 2 && twin_wgs <= 2 * (uint64_t)c->cus) return TV_KERNEL_TWIN;
    return n <= 32768 ? TV_KERNEL_SPLIT : TV_KERNEL_LANE;
}

// Kernel of a launch over the whole shard.
int choose_kernel(const tv_ctx* c) {
    const uint64_t last = c->P - 1;
    const bool short_last = last >= c->first && last < c->first + c->count && piece_len(c, last) != c->L;
    return choose_kernel_n(c, c->count, short_last);
}

// The lane kernel's loads for a launch of n pieces: pairs once every SIMD holds a wave (>= 64 lanes x 4 SIMDs x
// CUs pieces; TV_OPT_LANE_PAIRS overrides).
uint32_t lane_pairs_for(const tv_ctx* c, uint64_t n) {
    if (c->lane_pairs == 1) return 1;
    if (c->lane_pairs == 2) return 0;
    return n >= 256ull * (uint64_t)c->cus ? 1u : 0u;
}

// One launch over the resident shard with the chosen kernel (TV_OPT_TWIN_PACK: on the CU-masked pack_stream,
// forked after everything queued on c->stream and joined back into it).
int launch_resident(tv_ctx* c, const TvPieces& p_in, int kernel, bool hash) {
    TvPieces p = p_in;
    p.lane_pairs = lane_pairs_for(c, p.n);
    // A CU running ONE 2-wave twin workgroup spends ~80 more shader cycles per block than one running two
    // (PMC GRBM_GUI_ACTIVE: 1,806 vs 1,727; sleeping fillers do not help, working ones do: DESIGN.md section 5).
    // With fewer real workgroups than 2 per CU, companions fill the grid to 2 x CUs: they re-hash main
    // workgroups' pieces on otherwise idle SIMDs and discard the result (TV_OPT_TWIN_FILL, default on).
    if (kernel == TV_KERNEL_TWIN && c->twin_fill && !c->twin_pack && (c->split_pairs < 2 || c->split_pairs > 5)) {
        p.fill_to = 2u * (uint32_t)c->cus;
        p.fill_all = c->fill_all ? 1u : 0u;
    }
    if (kernel == TV_KERNEL_TWIN && c->twin_pack && (c->split_pairs < 2 || c->split_pairs > 5)) {
        // 2-wave twin workgroups, 60 KiB of LDS each: at most two per CU.  Fewer than 2 x CUs of them: mask
        // the launch to ceil(wgs / 2) CUs so that every busy CU holds two (TV_OPT_TWIN_PACK).
        const uint64_t wgs = (p.n_main + 31) / 32 + (p.n_main < p.n ? 1 : 0);
        const int k = (int)std::min<uint64_t>((uint64_t)c->cus, (wgs + 1) / 2);
        if (k < c->cus) {
            if (c->pack_cus != k) {
                if (c->pack_stream) TV_HIP(c, hipStreamDestroy(c->pack_stream));
                c->pack_stream = nullptr;
                c->pack_cus = 0;
                std::vector<uint32_t> m((c->cus + 31) / 32, 0);
                for (int i = 0; i < k; i++) m[i / 32] |= 1u << (i % 32);
                TV_HIP(c, hipExtStreamCreateWithCUMask(&c->pack_stream, (uint32_t)m.size(), m.data()));
                c->pack_cus = k;
            }
            TV_HIP(c, hipEventRecord(c->ev_fork, c->stream));
            TV_HIP(c, hipStreamWaitEvent(c->pack_stream, c->ev_fork, 0));
            TV_HIP(c, tv_launch_verify(p, kernel, hash, c->pack_stream, c->split_pairs, &c->last_workgroups));
            TV_HIP(c, hipEventRecord(c->ev_join, c->pack_stream));
            TV_HIP(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
            return TV_OK;
        }
    }
    TV_HIP(c, tv_launch_verify(p, kernel, hash, c->stream, c->split_pairs, &c->last_workgroups));
    return TV_OK;
}

TvPieces resident_launch(const tv_ctx* c) {
    TvPieces p{};
    p.data = c->d_payload;
    p.stride = c->stride;
    p.data_off = 0;
    p.L = c->L;
    p.n = (uint32_t)c->count;
    const uint64_t last = c->P - 1;
    p.last_idx = (last >= c->first && last < c->first + c->count) ? (uint32_t)(last - c->first) : 0xFFFFFFFFu;
    p.last_len = piece_len(c, last);
    // a short last piece hashes in a group of its own: in a main group its short tail would put every
    // other lane of the group on the slow padded-block path for the rest of the piece
    p.n_main = (p.last_idx != 0xFFFFFFFFu && p.last_len != c->L) ? p.n - 1 : p.n;
    p.blk_begin = 0;
    p.blk_end = UINT64_MAX;
    p.finalize = 1;
    p.dcount = (uint32_t)c->count;
    p.state = c->d_state;
    p.digests = c->d_digests;
    p.avail64 = c->d_base_avail;
    p.out64 = c->d_out;
    p.out_digests = c->d_hash;
    p.clock = c->clock_probe ? c->d_clock : nullptr;
    return p;
}

// ---- what the resident payload holds: the whole shard, the open window, or a slot pool ---------------------

// Shard-relative pieces [*j0, *j0 + *n) whose bytes the payload can take now: the shard; a windowed layout's
// open window (n = 0 when none is open); a slot pool's whole shard (any piece may take a free slot).
void resident_pieces(const tv_ctx* c, uint64_t* j0, uint64_t* n) {
    *j0 = 0;
    *n = c->count;
    if (c->win) {
        if (c->win_cur == UINT64_MAX) {
            *n = 0;
            return;
        }
        *j0 = c->win_cur * c->win_n;
        *n = std::min(c->win_n, c->count - *j0);
    }
}

uint8_t* win_base(const tv_ctx* c, int buf) { return c->d_payload + (uint64_t)buf * c->win_buf_bytes; }

// Device address of GLOBAL piece i's byte 0 (i among the resident pieces).  A slot pool gives the piece its
// slot, taking a free one the first time (TV_ERR_STATE when every slot holds a piece not yet listed).
int piece_dst(tv_ctx* c, uint64_t i, uint8_t** out) {
    const uint64_t j = i - c->first;
    if (c->slots) {
        auto it = c->slot_of.find(j);
        if (it == c->slot_of.end()) {
            if (c->slot_free.empty())
                return fail(c, TV_ERR_STATE,
                            "every one of the %llu slots (TV_OPT_LIST_SLOTS) holds a staged piece not yet listed: "
                            "tv_verify_list them first", (unsigned long long)c->slots);
            it = c->slot_of.emplace(j, c->slot_free.back()).first;
            c->slot_free.pop_back();
        }
        *out = c->d_payload + (uint64_t)it->second * c->stride;
    } else if (c->win) {
        *out = win_base(c, c->win_buf) + (j - c->win_cur * c->win_n) * c->stride;
    } else {
        *out = c->d_payload + j * c->stride;
    }
    return TV_OK;
}

// The same for reading (tv_read): a slot pool's piece must hold a slot.
int piece_src(tv_ctx* c, uint64_t i, const uint8_t** out) {
    if (c->slots && !c->slot_of.count(i - c->first))
        return fail(c, TV_ERR_STATE, "piece %llu holds no slot (it was never staged, or was listed since)",
                    (unsigned long long)i);
    uint8_t* p = nullptr;
    const int rc = piece_dst(c, i, &p);
    *out = p;
    return rc;
}

// One launch over shard pieces [j0, j0 + n) whose bytes start at `data` (a window buffer): the resident
// geometry narrowed to them; digest, state and hash rows are the shard's (dcount = count), offset by j0.
TvPieces window_launch(const tv_ctx* c, uint64_t j0, uint64_t n, const uint8_t* data) {
    TvPieces p = resident_launch(c);
    p.data = data;
    p.n = (uint32_t)n;
    const uint64_t last = c->P - 1, g0 = c->first + j0;
    p.last_idx = (last >= g0 && last < g0 + n) ? (uint32_t)(last - g0) : 0xFFFFFFFFu;
    p.n_main = (p.last_idx != 0xFFFFFFFFu && p.last_len != c->L) ? p.n - 1 : p.n;
    p.state = c->d_state + j0;
    p.digests = c->d_digests + j0;
    p.out_digests = c->d_hash + j0;
    p.avail64 = nullptr;
    p.out64 = nullptr;
    return p;
}

// ---- windowed layouts (the shard's payload exceeds TV_OPT_RESIDENT_BUDGET) ----------------------------------
//
// Window w = shard pieces [w*win_n, (w+1)*win_n).  Staging opens the window of the bytes it stages (win_enter);
// opening window w hashes the window open before it (win_seal: a HASH launch into the shard's digest rows d_hash,
// after the copies queued into its buffer) and its buffer's next copies wait for the kernel that last read it, so
// window w + 1 stages while window w hashes.  A pass ends at tv_verify / tv_hash (win_finalize), which then
// compare / read d_hash for the whole shard; staging after that starts a new pass.  Windows a pass never opens
// are never staged: their digests are zeroed (bit 0, zero digests), never a stale buffer's hash.

int zero_hash(tv_ctx* c, uint64_t j0, uint64_t j1) {
    if (j1 <= j0) return TV_OK;
    for (int k = 0; k < 5; k++)
        TV_HIP(c, hipMemsetAsync(c->d_hash + (uint64_t)k * c->count + j0, 0, (j1 - j0) * 4, c->stream));
    return TV_OK;
}

int win_pass_timing(tv_ctx* c) {
    if (!c->win_timing) {
        TV_HIP(c, hipEventRecord(c->ev_call0, c->stream));
        c->win_timing = true;
    }
    return TV_OK;
}

// Hash the open window (no-op when none is open).
int win_seal(tv_ctx* c) {
    if (c->win_cur == UINT64_MAX) return TV_OK;
    const uint64_t j0 = c->win_cur * c->win_n, n = std::min(c->win_n, c->count - j0);
    for (int l = 0; l < 2; l++) {  // after every copy queued into the buffer, on either staging lane
        TV_HIP(c, hipEventRecord(c->win_cp[l], lane_stream(c, l)));
        TV_HIP(c, hipStreamWaitEvent(c->stream, c->win_cp[l], 0));
    }
    if (c->win_launched == 0) TV_HIP(c, hipEventRecord(c->ev_k0, c->stream));
    const TvPieces p = window_launch(c, j0, n, win_base(c, c->win_buf));
    const int kernel = choose_kernel_n(c, n, p.n_main < p.n);
    const int rc = launch_resident(c, p, kernel, /*hash=*/true);
    if (rc) return rc;
    TV_HIP(c, hipEventRecord(c->win_ev[c->win_buf], c->stream));
    c->last_kernel = kernel;
    c->win_launched++;
    c->win_valid = j0 + n;
    c->win_cur = UINT64_MAX;
    return TV_OK;
}

// Open window w for staging.  A window of this pass already hashed is TV_ERR_STATE: staging ascends.
int win_enter(tv_ctx* c, uint64_t w) {
    if (c->win_done) {  // the last pass was finalized: this stage starts a new one
        c->win_done = false;
        c->win_valid = 0;
        c->win_launched = 0;
        c->win_timing = false;
    }
    if (w == c->win_cur) return TV_OK;
    if ((c->win_cur != UINT64_MAX && w < c->win_cur) || w * c->win_n < c->win_valid)
        return fail(c, TV_ERR_STATE,
                    "windowed layout (the shard's %llu pieces exceed the device budget; windows of %llu pieces): "
                    "pieces %llu.. were already hashed this pass -- stage in ascending piece order, or call "
                    "tv_verify / tv_hash to end the pass first", (unsigned long long)c->count,
                    (unsigned long long)c->win_n, (unsigned long long)(c->first + w * c->win_n));
    int rc = win_pass_timing(c);
    if (!rc) rc = win_seal(c);
    if (!rc) rc = zero_hash(c, c->win_valid, w * c->win_n);   // windows skipped over: never staged
    if (rc) return rc;
    c->win_valid = w * c->win_n;
    c->win_buf = (c->win_buf + 1) % c->win_bufs;
    // the buffer is free once the kernel that last read it is done (copies on either lane wait for it; fills and
    // kernels follow it on the compute stream)
    TV_HIP(c, hipStreamWaitEvent(c->copy_stream, c->win_ev[c->win_buf], 0));
    TV_HIP(c, hipStreamWaitEvent(c->copy_stream2, c->win_ev[c->win_buf], 0));
    c->win_cur = w;
    return TV_OK;
}

// End the pass: hash the open window, zero the windows never opened; d_hash then holds the whole shard.
int win_finalize(tv_ctx* c) {
    if (c->win_done) return TV_OK;
    int rc = win_pass_timing(c);
    if (!rc) rc = win_seal(c);
    if (rc) return rc;
    if (c->win_launched == 0) TV_HIP(c, hipEventRecord(c->ev_k0, c->stream));
    rc = zero_hash(c, c->win_valid, c->count);
    if (rc) return rc;
    c->win_valid = c->count;
    TV_HIP(c, hipEventRecord(c->ev_k1, c->stream));
    c->win_done = true;
    c->win_passes++;
    return TV_OK;
}

// The window of shard-relative piece j.
inline uint64_t win_of(const tv_ctx* c, uint64_t j) { return j / c->win_n; }

// Linear byte where window w's pieces end (the next window's first byte; the shard's end for the last one).
uint64_t win_end_linear(const tv_ctx* c, uint64_t w) {
    const uint64_t j1 = std::min(c->count, (w + 1) * c->win_n);
    const uint64_t last = c->first + j1 - 1;
    return last * c->L + piece_len(c, last);
}

// The state every non-stream call needs.  need_resident: the call reads or writes the resident payload
// (absent with TV_OPT_RESIDENT = 0).  Calls sharing the output / chunk buffers wait for a stream to end.
int require_layout(tv_ctx* c, bool need_digests, bool need_resident = false) {
    if (!c->has_layout) return fail(c, TV_ERR_STATE, "tv_set_layout has not been called");
    if (need_digests && !c->digests_set) return fail(c, TV_ERR_STATE, "tv_set_digests has not been called");
    if (c->st.active) return fail(c, TV_ERR_STATE, "a stream is active (finish it with tv_stream_end or tv_stream_abort)");
    if (need_resident && c->count && !c->d_payload)
        return fail(c, TV_ERR_STATE, "no resident payload (the layout was set with TV_OPT_RESIDENT = 0): use tv_stream_*");
    return TV_OK;
}

int read_bits(tv_ctx* c, uint8_t* out) {
    const size_t nbytes = (c->count + 7) / 8;
    int rc = ensure_hbits(c, c->bit_words * 8);
    if (rc) return rc;
    TV_HIP(c, hipMemcpyAsync(c->h_bits, c->d_out, c->bit_words * 8, hipMemcpyDeviceToHost, c->stream));
    TV_HIP(c, hipEventRecord(c->ev_call1, c->stream));
    TV_HIP(c, hipEventSynchronize(c->ev_call1));
    memcpy(out, c->h_bits, nbytes);
    if (c->count % 8) out[nbytes - 1] &= (uint8_t)(0xFF00u >> (c->count % 8));  // spare bits 0
    return TV_OK;
}

int finish_timing(tv_ctx* c) {
    TV_HIP(c, hipEventElapsedTime(&c->kernel_ms, c->ev_k0, c->ev_k1));
    TV_HIP(c, hipEventElapsedTime(&c->total_ms, c->ev_call0, c->ev_call1));
    return TV_OK;
}

// Host memcpy into a pinned ring slot, split over up to `threads` threads in 4 MiB parts when it is
// long (one core copies pageable memory at well under the PCIe rate).
void copy_into_ring(Pool& pool, uint8_t* dst, const uint8_t* src, uint64_t n, int threads) {
    constexpr uint64_t kPart = 4ull << 20;
    const uint64_t parts = (n + kPart - 1) / kPart;
    pool.run(threads, parts, [&](uint64_t q) {
        const uint64_t o = q * kPart;
        tv_copy_host(dst + o, src + o, std::min(kPart, n - o));
    });
}

// Gather k rows of `width` bytes at pitch `pitch` from src into dst (packed at pitch width), on up to
// `threads` threads.
void gather_rows(Pool& pool, uint8_t* dst, const uint8_t* src, uint64_t width, uint64_t pitch, uint64_t k,
                 int threads) {
    const uint64_t per = std::max<uint64_t>(1, (4ull << 20) / std::max<uint64_t>(1, width));  // rows per task
    const uint64_t tasks = (k + per - 1) / per;
    pool.run(threads, tasks, [&](uint64_t q) {
        for (uint64_t r = q * per; r < std::min(k, (q + 1) * per); r++) tv_copy_host(dst + r * width, src + r * pitch, width);
    });
}

// One host -> device copy on the lane's copy stream, dword-aligned.  The DMA engine moves 1-byte-aligned
// data ~10x slower than dword-aligned data (57 vs 5.7 GB/s, tools/dma_align_probe.py): when src and
// dst agree mod 4, the 0-3 byte head and tail go as separate tiny copies and the body is aligned.
int dma_h2d(tv_ctx* c, uint8_t* dst, const uint8_t* src, uint64_t n, int lane = 0) {
    hipStream_t cs = lane_stream(c, lane);
    const uint64_t mis = (uintptr_t)dst & 3;
    if (n >= 64 && mis == ((uintptr_t)src & 3) && (mis || (n & 3))) {
        const uint64_t head = (4 - mis) & 3, body = (n - head) & ~3ull, tail = n - head - body;
        if (head) TV_HIP(c, hipMemcpyAsync(dst, src, head, hipMemcpyHostToDevice, cs));
        TV_HIP(c, hipMemcpyAsync(dst + head, src + head, body, hipMemcpyHostToDevice, cs));
        if (tail) TV_HIP(c, hipMemcpyAsync(dst + head + body, src + head + body, tail, hipMemcpyHostToDevice, cs));
        return TV_OK;
    }
    TV_HIP(c, hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, cs));
    return TV_OK;
}

// Stage one contiguous range of LINEAR bytes that lies inside a single piece or covers whole
// pieces; src is host memory.  Rows of whole pieces use one 2D copy (src pitch L, dst pitch stride).
// A page-locked src is read by DMA directly; pageable memory is copied through the lane's pinned ring.
// `src_in_ring`: src already lies in one of the lane's ring slots (tv_stage_files' packed reads, the
// cold-window preads).  Such a source is never bounced through the ring again: the bounce would take the
// ring's next slots, and after kRingSlots takes that is the very slot being read (its event is recorded
// only after these copies are queued), so the bounce would overwrite bytes still to be copied.  The
// slot bytes sit at their LINEAR offset's alignment mod 4, which is the destination's whenever L % 4 == 0
// (every power-of-two piece length); with other L the copy is simply not dword-aligned.
int stage_copy(tv_ctx* c, uint64_t pos, const uint8_t* src, uint64_t n, bool pinned, int lane = 0,
               bool src_in_ring = false) {
    hipStream_t cs = lane_stream(c, lane);
    while (n) {
        const uint64_t i = pos / c->L, within = pos % c->L;
        const uint64_t plen = piece_len(c, i);
        uint8_t* dst = nullptr;
        {
            const int rc = piece_dst(c, i, &dst);  // (a slot pool gives piece i its slot here)
            if (rc) return rc;
        }
        dst += within;
        const bool whole = within == 0 && plen == c->L && n >= c->L;
        // A pinned source whose alignment cannot match the destination's (mod 4; whole-piece rows need
        // it at 0 mod 4 and L % 4 == 0) goes through the ring instead: one memcpy, then aligned DMA.
        // (TV_OPT_DEBUG_REBOUNCE re-enables the bounce for ring-resident sources: the slot lease then
        // keeps the source slot out of the bounce's reach.)
        const bool via_ring = (!src_in_ring || c->debug_rebounce) &&
                              (!pinned || (whole ? (((uintptr_t)src & 3) != 0 && c->L % 4 == 0)
                                                 : (((uintptr_t)src ^ (uintptr_t)dst) & 3) != 0));
        const uint64_t cap = via_ring ? (uint64_t)kRingSlotBytes - 4 : UINT64_MAX;
        SlotLease slot(c, lane);
        if (via_ring) {
            int rc = slot.take();
            if (rc) return rc;
        }
        uint64_t bytes;
        if (whole && c->L <= cap) {
            // k whole pieces (none of them the short last piece): one 2D copy, rows at pitch L -> stride
            uint64_t k = std::min<uint64_t>(n / c->L, cap / c->L);
            const uint64_t last_full = (c->total % c->L) ? c->P - 1 : c->P;  // first index that is not full
            k = std::min<uint64_t>(k, (last_full > i) ? last_full - i : 1);
            if (c->slots) k = 1;  // a slot pool's rows are not consecutive pieces
            bytes = k * c->L;
            const uint8_t* from = via_ring ? slot.ptr() : src;
            if (via_ring) copy_into_ring(c->pool[lane], slot.ptr(), src, bytes, c->file_threads);
            TV_HIP(c, hipMemcpy2DAsync(dst, c->stride, from, c->L, c->L, k, hipMemcpyHostToDevice, cs));
        } else {
            bytes = std::min<uint64_t>({n, plen > within ? plen - within : 0, cap});
            if (bytes == 0) return fail(c, TV_ERR_ARG, "stage offset %llu is past piece %llu", (unsigned long long)pos,
                                        (unsigned long long)i);
            const uint8_t* from = src;
            if (via_ring) {  // place the bytes at the destination's alignment inside the slot
                uint8_t* r = slot.ptr() + ((uintptr_t)dst & 3);
                copy_into_ring(c->pool[lane], r, src, bytes, c->file_threads);
                from = r;
            }
            int rc = dma_h2d(c, dst, from, bytes, lane);
            if (rc) return rc;
        }
        if (via_ring) {
            int rc = slot.release();
            if (rc) return rc;
        }
        pos += bytes;
        src += bytes;
        n -= bytes;
    }
    return TV_OK;
}

// Every exit of a call that queued copies from caller memory drains its copy lane (and, unless `compute` is
// false, the compute stream), so no DMA still reads the caller's buffer after the call returns (also on error
// paths), and destroys the call's own events.  Staging calls leave the compute stream running: a windowed
// layout's window kernel then hashes on while the caller reads the next bytes.
struct DrainGuard {
    tv_ctx* c;
    int lane;
    bool compute;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    explicit DrainGuard(tv_ctx* ctx, int copy_lane = 0, bool sync_compute = true)
        : c(ctx), lane(copy_lane), compute(sync_compute) {}
    ~DrainGuard() {
        (void)hipStreamSynchronize(lane_stream(c, lane));
        if (compute) (void)hipStreamSynchronize(c->stream);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        (void)hipGetLastError();
    }
    DrainGuard(const DrainGuard&) = delete;
    DrainGuard& operator=(const DrainGuard&) = delete;
};

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr{};
    const bool ok = hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type == hipMemoryTypeHost &&
                    attr.devicePointer != nullptr;
    (void)hipGetLastError();
    return ok;
}

// Clip the LINEAR range [off, off + len) to this ctx's shard: [*a, *b) (empty when *a >= *b).
void clip_to_whole_shard(const tv_ctx* c, uint64_t off, uint64_t len, uint64_t* a, uint64_t* b) {
    const uint64_t lo = c->first * c->L;
    const uint64_t last = c->first + c->count - 1;
    const uint64_t hi = last * c->L + piece_len(c, last);
    *a = std::max(off, lo);
    *b = std::min(off + len, hi);
}

// Clip it to the pieces the payload can take now (resident_pieces: the shard, or a windowed layout's open window).
void clip_to_shard(const tv_ctx* c, uint64_t off, uint64_t len, uint64_t* a, uint64_t* b) {
    uint64_t j0, n;
    resident_pieces(c, &j0, &n);
    if (n == 0) {
        *a = *b = 0;
        return;
    }
    const uint64_t lo = (c->first + j0) * c->L;
    const uint64_t last = c->first + j0 + n - 1;
    const uint64_t hi = last * c->L + piece_len(c, last);
    *a = std::max(off, lo);
    *b = std::min(off + len, hi);
}

// A later call that stages every byte of a piece clears its unreadable mark (recover_segment's), so a repaired
// file re-staged into the same layout reads again: the whole pieces inside LINEAR [a, b).
void clear_bad(tv_ctx* c, uint64_t a, uint64_t b) {
    if (!c->any_file_bad || b <= a || c->count == 0) return;
    const uint64_t lo = c->first * c->L;
    if (b <= lo) return;
    uint64_t i = std::max(a, lo);
    i = (i + c->L - 1) / c->L;  // the first piece starting at or after a
    for (; i < c->first + c->count && i * c->L + piece_len(c, i) <= b; i++) {
        const uint64_t j = i - c->first;
        c->file_bad[j >> 3] &= (uint8_t)~(0x80u >> (j & 7));
    }
}

// Queue the copies of LINEAR bytes [a, b) (inside the shard) on the copy stream; byte `pos` is read
// from base + (pos - base_off).  Pieces are split at piece boundaries (a piece is shorter than L only
// at the end of the torrent, piece.ts:16-19); bytes in a short last piece's missing tail are skipped.
int stage_range(tv_ctx* c, uint64_t a, uint64_t b, const uint8_t* base, uint64_t base_off, bool pinned,
                int lane = 0, bool src_in_ring = false) {
    uint64_t pos = a;
    while (pos < b) {
        const uint64_t i = pos / c->L, within = pos % c->L;
        const uint64_t plen = piece_len(c, i);
        if (within >= plen) {  // inside a short last piece's missing tail: nothing to store
            pos = (i + 1) * c->L;
            continue;
        }
        uint64_t n;
        if (within == 0 && plen == c->L) {
            n = ((b - pos) / c->L) * c->L;  // whole pieces
            if (n == 0) n = b - pos;
        } else {
            n = std::min(b - pos, plen - within);
        }
        int rc = stage_copy(c, pos, base + (pos - base_off), n, pinned, lane, src_in_ring);
        if (rc) return rc;
        pos += n;
    }
    return TV_OK;
}

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

int stream_begin_locked(tv_ctx* c, const uint8_t* avail_bits) {
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
    } else {               // columns across the whole shard
        st.C = stream_column(c);
        st.wn = c->count;
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
    st.rows_per_req = std::max<uint64_t>(1, kRingSlotBytes / st.C);
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

}  // namespace

// ============================================================================================
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
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->win_ev[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->win_cp[k], hipEventDisableTiming);
    }
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
    free_device(c);
    for (int s = 0; s < kRingSlots; s++) {
        if (c->ring[s]) (void)hipHostFree(c->ring[s]);
        if (c->ring_ev[s]) (void)hipEventDestroy(c->ring_ev[s]);
        if (c->ring2[s]) (void)hipHostFree(c->ring2[s]);
        if (c->ring2_ev[s]) (void)hipEventDestroy(c->ring2_ev[s]);
    }
    if (c->h_bits) (void)hipHostFree(c->h_bits);
    if (c->d_clock) (void)hipFree(c->d_clock);
    for (hipEvent_t ev : {c->ev_call0, c->ev_k0, c->ev_k1, c->ev_call1, c->ev_avail, c->col_ev[0], c->col_ev[1],
                          c->done_ev[0], c->done_ev[1], c->ev_fork, c->ev_join, c->win_ev[0], c->win_ev[1],
                          c->win_cp[0], c->win_cp[1]})
        if (ev) (void)hipEventDestroy(ev);
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
            if (value < 0 || value > 2) return fail(c, TV_ERR_ARG, "TV_OPT_TWIN_FILL must be 0, 1 or 2");
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
    c->win = false;
    c->win_n = 0;
    c->win_bufs = 0;
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
    // GPU of any free memory).  A failed allocation is retried at half the budget: only the windows shrink.
    for (;;) {
        if (need_payload && !c->slots && need_payload > budget) {
            uint64_t bufs = 2, W = budget / 2 > kSlack ? (budget / 2 - kSlack) / c->stride : 0;
            if (W == 0) {
                bufs = 1;
                W = budget > kSlack ? (budget - kSlack) / c->stride : 0;
            }
            W = std::max<uint64_t>(1, std::min(W, shard_count));  // (one piece larger than the budget: held anyway)
            if (W >= 256) W = W / 64 * 64;                        // whole 64-piece waves per window
            c->win = true;
            c->win_n = W;
            c->win_bufs = (int)bufs;
            c->win_buf_bytes = W * c->stride + kSlack;
            need_payload = bufs * c->win_buf_bytes;
        }
        // (an allocation larger than the budget is never kept: the budget bounds what the ctx holds)
        if (!need_payload || !reuse_fits(need_payload, c->cap_payload) || (budget && c->cap_payload > budget))
            free_payload(c);
        if (!need_payload || c->d_payload) break;
        const hipError_t e = hipMalloc((void**)&c->d_payload, need_payload);
        if (e == hipSuccess) {
            c->cap_payload = need_payload;
            c->n_payload_allocs++;
            c->n_device_allocs++;
            break;
        }
        (void)hipGetLastError();
        c->d_payload = nullptr;
        if (e != hipErrorOutOfMemory || c->slots || need_payload <= (64ull << 20))
            return fail(c, e == hipErrorOutOfMemory ? TV_ERR_NOMEM : TV_ERR_HIP, "hipMalloc(%llu) of the payload: %s",
                        (unsigned long long)need_payload, hipGetErrorString(e));
        budget = need_payload / 2;  // windows of half the size
        need_payload = shard_count * c->stride + kSlack;
        c->win = false;
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

}  // extern "C"

namespace {

// tv_stage's work with the lock held and the arguments checked: LINEAR [linear_offset, linear_offset + len) from
// src queued on the copy lane (window by window on a windowed layout).  The caller drains the lane (DrainGuard),
// synchronises it to see copy failures and then clears the staged pieces' marks (clear_staged).
int stage_locked(tv_ctx* c, uint64_t linear_offset, const uint8_t* src, uint64_t len) {
    uint64_t a, b;
    clip_to_whole_shard(c, linear_offset, len, &a, &b);
    if (a >= b) return TV_OK;
    const bool pinned = is_pinned(src);
    if (!c->win) return stage_range(c, a, b, src, linear_offset, pinned);
    // window by window, ascending: opening the next window hashes the previous one (win_enter)
    for (uint64_t pos = a; pos < b;) {
        const uint64_t w = win_of(c, pos / c->L - c->first);
        int rc = win_enter(c, w);
        if (rc) return rc;
        uint64_t wa, wb;
        clip_to_shard(c, pos, b - pos, &wa, &wb);
        if (wa < wb) {
            rc = stage_range(c, wa, wb, src, linear_offset, pinned);
            if (rc) return rc;
        }
        pos = win_end_linear(c, w);
    }
    return TV_OK;
}

void clear_staged(tv_ctx* c, uint64_t linear_offset, uint64_t len) {
    uint64_t a, b;
    clip_to_whole_shard(c, linear_offset, len, &a, &b);
    clear_bad(c, a, b);
}

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

namespace {

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
        if (kernel == TV_KERNEL_TWIN && (c->twin_fill == 2 || (c->twin_fill == 1 && list_wgs >= (uint64_t)c->cus))) {
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
    DrainGuard drain(c);  // no DMA reads the caller's buffer after the call returns, also on error paths
    rc = stream_begin_locked(c, av.data());
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

namespace {

// Public stream calls: a HIP failure leaves the stream unusable, so it is aborted (the ctx stays usable).
int stream_result(tv_ctx* c, int rc) {
    if (rc == TV_ERR_HIP || rc == TV_ERR_NOMEM) stream_abort_locked(c);
    return rc;
}

}  // namespace

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
        case TV_COUNTER_BUDGET: *value = c->budget; return TV_OK;
        case TV_COUNTER_SLOTS_USED: *value = c->slot_of.size(); return TV_OK;
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
