// tv_ctx.h -- internal to libtorrent_verify.so: the context (struct tv_ctx, one per GPU) and the helpers its
// translation units share.  tv_context.hip: lifecycle, options, layout, digests, counters; tv_core.hip: errors, NUMA,
// staging rings, windows, slot pool, kernel choice, the host -> HBM copy path; tv_stage.hip: staging from memory;
// tv_files.hip: staging from files; tv_stream.hip: the streamed engine; tv_verify.hip: verify / list / hash.
// Nothing here is exported (the link exports tv_* only: exports.map).
#pragma once
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/torrent_verify.h"
#include "tv_host.h"
#include "tv_internal.h"
#include "tv_options_internal.h"
#include "tv_plan.h"

namespace tvi {

constexpr uint64_t kSlack = 256;                          // bytes past the last resident piece (tail over-read)
constexpr int kRingSlots = TV_STREAM_RING_SLOTS;          // pinned staging buffers per lane
constexpr size_t kRingSlotBytes = TV_STREAM_SLOT_BYTES;
constexpr int kWinHashStreams = 4;                        // hash streams of a windowed layout, at most

// Pin the calling thread to `cpus` (nullptr: leave it).  Used for the library's own threads only.
void pin_thread(const cpu_set_t* cpus);

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

// A cold-read bounce buffer (TV_OPT_FILE_BOUNCE): kBounceBytes of page-locked memory and the event of the DMA that
// last read it.
constexpr uint64_t kBounceBytes = 4ull << 20;
struct Bounce {
    uint8_t* ptr = nullptr;
    hipEvent_t ev = nullptr;
    bool recorded = false;
};

}  // namespace tvi

using tvi::kRingSlots;
using tvi::Pool;
using tvi::StreamState;

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
    bool file_direct = false;            // TV_OPT_FILE_DIRECT: long segments DMA'd from registered page-cache pages
    bool file_concurrent = true;         // tv_stage_files: long segments on two staging lanes
    int file_odirect = 1;                // TV_OPT_FILE_ODIRECT: cold chunks read with O_DIRECT (2: its reads fail, tests)
    int file_bounce = 2;                 // TV_OPT_FILE_BOUNCE: cold O_DIRECT reads into small reused page-locked buffers
    uint64_t stream_cold_window = 0;     // TV_OPT_STREAM_COLD_WINDOW (0: 512 pieces)
    int stream_cold_readers = 0;         // TV_OPT_STREAM_COLD_READERS (0: 2 x file_threads)
    uint64_t stream_cold_req = 0;        // TV_OPT_STREAM_COLD_REQ (0: one ring slot)
                                         // DMA'd from there (readers per lane), 0 = into the ring's 64 MiB slots
    uint64_t file_direct_min = 32ull << 20;  // tv_stage_files: segments >= this take the tv_stage_file path
    int file_threads = 16;                   // tv_stage_files: reader threads
    bool resident = true;                    // TV_OPT_RESIDENT
    bool debug_rebounce = false;             // TV_OPT_DEBUG_REBOUNCE
    bool twin_pack = false;                  // TV_OPT_TWIN_PACK
    int twin_fill = 1;                       // TV_OPT_TWIN_FILL: 0 off, 1 auto, 2 also on short lists, 3 on always
    uint32_t kfd_gpu_id = 0;                 // the GPU's KFD id (co-tenant check of the companions; 0 = unknown)
    long create_pid = 0;                     // getpid() at tv_create (a forked child makes no co-tenant probe)
    bool cotenant_checked = false;           // cotenant_bytes is fresh (read at cotenant_at)
    uint64_t cotenant_bytes = 0;             // this GPU's memory other processes hold (KFD accounting)
    std::chrono::steady_clock::time_point cotenant_at;
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
    // windowed layouts: shard-relative MSB-first bits of the pieces in windows this pass never staged (their d_hash
    // rows are zeroed, never hashed): tv_verify reports them 0 even where an expected digest is 20 zero bytes
    std::vector<uint8_t> unhashed;
    bool any_unhashed = false;

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
    // cold-read bounce buffers of lane 0 / lane 1 (TV_OPT_FILE_BOUNCE), handed to the lane's readers from a free list
    std::vector<tvi::Bounce> bounce[2];
    std::vector<int> bounce_free[2];
    std::mutex bounce_mu[2];
    std::condition_variable bounce_cv[2];
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
    int win_bufs = 0;                  // buffers in d_payload (window k + 1 stages while those before it hash)
    uint64_t win_buf_bytes = 0;        // bytes per buffer (win_n * stride + kSlack)
    uint64_t win_cur = UINT64_MAX;     // window open for staging (UINT64_MAX: none)
    int win_buf = 1;                   // its buffer
    uint64_t win_valid = 0;            // shard pieces [0, win_valid) are hashed (or zeroed: never staged) this pass
    bool win_done = false;             // the pass is finalized: d_hash holds every shard piece's digest
    bool win_timing = false;           // ev_call0 / ev_k0 recorded for this pass
    uint64_t win_launched = 0;         // windows hashed this pass
    uint64_t win_passes = 0;           // passes finalized since tv_set_layout
    hipEvent_t win_ev[tvi::kWinBufsMax] = {};   // the last kernel reading buffer k
    hipEvent_t win_cp[2] = {nullptr, nullptr};  // copies into the window queued on lane k (kernel waits on them)
    // Hash streams: window w hashes on the compute stream when w mod win_nhs == 0, else on win_hs[w mod win_nhs - 1]
    // (companions off there), so up to win_nhs windows hash side by side while the next ones stage; win_nhs = 1: every
    // window on the compute stream (the rounds 4-5 form).  win_hs[0] is created by tv_create right after the compute
    // stream (its own hardware queue where HIP has one free), the others when a layout needs them.
    int win_bufs_opt = 0;              // TV_OPT_WIN_BUFS (0: tv_plan.h kWinBufsDefault)
    int win_streams_opt = 0;           // TV_OPT_WIN_STREAMS (0: win_bufs - 1, at most kWinHashStreams)
    int win_nhs = 1;                   // hash streams of the current windowed layout, the compute stream included
    hipStream_t win_hs[tvi::kWinHashStreams - 1] = {};
    hipEvent_t win_hs_ev[tvi::kWinHashStreams - 1] = {};  // joins a hash stream into the compute stream

    // Slot pool (TV_OPT_LIST_SLOTS = K): the payload holds K piece slots instead of the shard; a staged piece
    // takes a slot until tv_verify_list lists it (incremental verify).
    uint64_t list_slots_opt = 0;
    uint64_t slots = 0;                // slots of the current layout (0: not a slot layout)
    std::unordered_map<uint64_t, uint32_t> slot_of;  // shard-relative piece -> slot
    std::vector<uint32_t> slot_free;
    std::mutex slot_mu;                // piece_dst's slot path: tv_stage_files' lane-1 helper stages beside the caller

    bool open_rw = true;               // TV_OPT_OPEN_RW: files opened read + write (fsStorage.get) or read-only
    bool stream_rows = false;          // TV_OPT_STREAM_ROWS: stream requests carry whole pieces (windows of pieces)
    int lane_pairs = 0;                // TV_OPT_LANE_PAIRS: 0 auto (>= 256 x CUs pieces in the launch), 1 on, 2 off
    bool clock_probe = false;          // TV_OPT_CLOCK_PROBE: verify / hash launches stamp their clock into d_clock
    uint64_t* d_clock = nullptr;       // {shader clock, real-time} counters at the start and end of workgroup 0
    cpu_set_t proc_cpus;               // the process's CPUs at tv_create (what "unpinned" workers run on)
    std::atomic<uint64_t> file_ns[TV_FILE_CLOCK_N] = {};  // the file staging phase clock (tv_options_internal.h)
    bool proc_cpus_ok = false;
};

namespace tvi {

// ---- errors ---------------------------------------------------------------------------------------------------

// Record the message (on the ctx and the calling thread) and return `code`.
int fail(tv_ctx* c, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
extern thread_local std::string g_thread_error;

#define TV_HIP(c, call)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail((c), e_ == hipErrorOutOfMemory ? TV_ERR_NOMEM : TV_ERR_HIP, "%s: %s (%s:%d)", #call, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                             \
    } while (0)

// ---- geometry ---------------------------------------------------------------------------------------------------

uint64_t piece_len(const tv_ctx* c, uint64_t i);  // piece.ts:16-19
inline void set_bit(uint8_t* bf, uint64_t i) { bf[i >> 3] |= (uint8_t)(0x80u >> (i & 7)); }
inline bool get_bit(const uint8_t* bf, uint64_t i) { return (bf[i >> 3] >> (7 - (i & 7))) & 1; }
// Clip the LINEAR range [off, off + len) to this ctx's shard / to the pieces the payload can take now.
void clip_to_whole_shard(const tv_ctx* c, uint64_t off, uint64_t len, uint64_t* a, uint64_t* b);
void clip_to_shard(const tv_ctx* c, uint64_t off, uint64_t len, uint64_t* a, uint64_t* b);
int require_layout(tv_ctx* c, bool need_digests, bool need_resident = false);

// ---- files (fsStorage.get's open rules) -------------------------------------------------------------------------

int access_ok(const char* path, bool rw);
int open_file(const char* path, bool rw, int* err);
double cached_fraction(int fd, uint64_t fo, uint64_t n);   // page-cache residency of file bytes, sampled (tv_files.hip)
int fs_openable(const char* path, bool rw);

// ---- NUMA placement and the host worker pools --------------------------------------------------------------------

int gpu_numa_node(int device);
bool node_cpus(int node, cpu_set_t* out);
hipError_t host_malloc_on_node(void** p, size_t bytes, int node);
int page_node(const void* p);
inline const cpu_set_t* numa_cpus(const tv_ctx* c) {  // where the library's threads run (nullptr: unpinned)
    return (c->numa_bind && c->numa_cpus_ok) ? &c->numa_cpus : nullptr;
}
void apply_numa(tv_ctx* c);

// ---- device allocations ------------------------------------------------------------------------------------------

void free_payload(tv_ctx* c);
void free_per_piece(tv_ctx* c);
void free_words(tv_ctx* c);
void free_chunks(tv_ctx* c);
void free_list(tv_ctx* c);
void free_device(tv_ctx* c);
bool reuse_fits(uint64_t need, uint64_t cap);

// ---- companion workgroups on a shared GPU (TV_OPT_TWIN_FILL) ----------------------------------------------------

// Another process holding this much of the GPU's memory makes it a co-tenant: TV_OPT_TWIN_FILL = 1 (auto) then
// launches no companion workgroups (they would take CUs the other process may be using).
constexpr uint64_t kCotenantBytes = 1ull << 30;
uint32_t kfd_gpu_id(int device);
uint32_t kfd_check_id(tv_ctx* c);
uint64_t cotenant_vram(tv_ctx* c);
bool companions_on(tv_ctx* c);
int ensure_hbits(tv_ctx* c, size_t bytes);

// ---- staging lanes: a copy stream and a ring of pinned slots each ---------------------------------------------------

// Staging lane `which`: 0 = copy_stream + ring, 1 = copy_stream2 + ring2.  Lane 1 is used only by
// tv_stage_files' helper thread, so the two lanes never share a ring slot or a stream.
struct RingRef {
    uint8_t** buf;
    hipEvent_t* ev;
    bool* lent;
    int* next;
};
inline RingRef ring_ref(tv_ctx* c, int which) {
    return which ? RingRef{c->ring2, c->ring2_ev, c->ring2_lent, &c->ring2_next}
                 : RingRef{c->ring, c->ring_ev, c->ring_lent, &c->ring_next};
}
inline hipStream_t lane_stream(const tv_ctx* c, int which) { return which ? c->copy_stream2 : c->copy_stream; }
int ensure_ring(tv_ctx* c, int which = 0);
int take_slot(tv_ctx* c, int* slot, int which = 0);
int release_slot(tv_ctx* c, int slot, int which = 0);

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

// Every exit of a call that queued copies from caller memory drains its copy lane (and, unless `compute` is
// false, the compute stream), so no DMA still reads the caller's buffer after the call returns (also on error
// paths), and destroys the call's own events.  Staging calls leave the compute stream running: a windowed
// layout's window kernel then hashes on while the caller reads the next bytes.
struct DrainGuard {
    tv_ctx* c;
    int lane;
    bool compute;
    bool lane_sync = true;   // false: a staging pass that hands its lane straight to the next window's pass (the copies
                             // read ring slots and bounce buffers, whose events order their reuse; the call's last
                             // pass drains)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    explicit DrainGuard(tv_ctx* ctx, int copy_lane = 0, bool sync_compute = true)
        : c(ctx), lane(copy_lane), compute(sync_compute) {}
    ~DrainGuard() {
        if (lane_sync) (void)hipStreamSynchronize(lane_stream(c, lane));
        if (compute) (void)hipStreamSynchronize(c->stream);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        (void)hipGetLastError();
    }
    DrainGuard(const DrainGuard&) = delete;
    DrainGuard& operator=(const DrainGuard&) = delete;
};

bool is_pinned(const void* p);
void copy_into_ring(Pool& pool, uint8_t* dst, const uint8_t* src, uint64_t n, int threads);
void gather_rows(Pool& pool, uint8_t* dst, const uint8_t* src, uint64_t width, uint64_t pitch, uint64_t k, int threads);
int dma_h2d(tv_ctx* c, uint8_t* dst, const uint8_t* src, uint64_t n, int lane = 0);
int stage_copy(tv_ctx* c, uint64_t pos, const uint8_t* src, uint64_t n, bool pinned, int lane = 0,
               bool src_in_ring = false);
int stage_range(tv_ctx* c, uint64_t a, uint64_t b, const uint8_t* base, uint64_t base_off, bool pinned, int lane = 0,
                bool src_in_ring = false);
int stage_locked(tv_ctx* c, uint64_t linear_offset, const uint8_t* src, uint64_t len);
void clear_staged(tv_ctx* c, uint64_t linear_offset, uint64_t len);
void clear_bad(tv_ctx* c, uint64_t a, uint64_t b);

// ---- availability, kernel choice, launches ------------------------------------------------------------------------

int upload_base_avail(tv_ctx* c);
int launch_avail(tv_ctx* c, const uint8_t* avail_bits, const uint64_t** out);
int choose_kernel_n(const tv_ctx* c, uint64_t n, bool short_last);
int choose_kernel(const tv_ctx* c);
uint32_t lane_pairs_for(const tv_ctx* c, uint64_t n);
int launch_resident(tv_ctx* c, const TvPieces& p_in, int kernel, bool hash, hipStream_t on = nullptr,
                    bool alone = true);
int win_sync_streams(tv_ctx* c);
TvPieces resident_launch(const tv_ctx* c);
TvPieces window_launch(const tv_ctx* c, uint64_t j0, uint64_t n, const uint8_t* data);
int read_bits(tv_ctx* c, uint8_t* out);
int finish_timing(tv_ctx* c);

// ---- what the payload holds: the shard, a window of it, or a slot pool ------------------------------------------------

void resident_pieces(const tv_ctx* c, uint64_t* j0, uint64_t* n);
uint8_t* win_base(const tv_ctx* c, int buf);
int piece_dst(tv_ctx* c, uint64_t i, uint8_t** out);
int piece_src(tv_ctx* c, uint64_t i, const uint8_t** out);
int win_enter(tv_ctx* c, uint64_t w);
int win_finalize(tv_ctx* c);
inline uint64_t win_of(const tv_ctx* c, uint64_t j) { return j / c->win_n; }  // the window of shard piece j
uint64_t win_end_linear(const tv_ctx* c, uint64_t w);

// ---- the streamed engine (tv_stream.hip) -----------------------------------------------------------------------------

void stream_abort_locked(tv_ctx* c);
uint64_t stream_chunk_need(const tv_ctx* c);

}  // namespace tvi
