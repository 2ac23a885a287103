// tv_core.hip -- the context's internals (tv_ctx.h): errors, the NUMA placement of host threads and pinned memory, the
// staging rings and their slot leases, the per-piece device rows, kernel choice and resident launches, the windowed
// layouts and the slot pool, and the host -> HBM copy path every staging call shares.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <dirent.h>

#include <cctype>
#include <chrono>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "tv_ctx.h"

namespace tvi {

thread_local std::string g_thread_error;


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


// The KFD gpu_id of HIP device `device` (the topology node whose PCI location matches; 0: not found or not
// readable).  /sys/class/kfd/kfd/topology/nodes/N/properties carries `domain` and `location_id` = bus << 8 |
// device << 3 | function.
static uint32_t kfd_topology_gpu_id(int device) {
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, (int)sizeof bdf, device) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    unsigned dom = 0, bus = 0, dev = 0, fn = 0;
    if (sscanf(bdf, "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4) return 0;
    const unsigned loc = (bus << 8) | (dev << 3) | fn;
    for (int node = 0; node < 256; node++) {
        char path[128];
        snprintf(path, sizeof path, "/sys/class/kfd/kfd/topology/nodes/%d/properties", node);
        FILE* f = fopen(path, "r");
        if (!f) {
            if (errno == ENOENT) break;   // past the last node (EPERM: a node this process may not see)
            continue;
        }
        char key[64];
        unsigned long long v = 0, l = ~0ull, d = ~0ull;
        while (fscanf(f, "%63s %llu", key, &v) == 2) {
            if (!strcmp(key, "location_id")) l = v;
            else if (!strcmp(key, "domain")) d = v;
        }
        fclose(f);
        if (l != loc || d != dom) continue;
        snprintf(path, sizeof path, "/sys/class/kfd/kfd/topology/nodes/%d/gpu_id", node);
        f = fopen(path, "r");
        unsigned id = 0;
        if (f) {
            if (fscanf(f, "%u", &id) != 1) id = 0;
            fclose(f);
        }
        return id;
    }
    return 0;
}

// vram_<gpu_id> of every process in KFD's accounting (pid as the kernel driver numbers it), sorted by pid.
static std::vector<std::pair<long, uint64_t>> kfd_vram(uint32_t gpu_id) {
    std::vector<std::pair<long, uint64_t>> out;
    if (DIR* d = opendir("/sys/class/kfd/kfd/proc")) {
        while (dirent* e = readdir(d)) {
            char* end = nullptr;
            const long pid = strtol(e->d_name, &end, 10);
            if (end == e->d_name || *end) continue;
            char path[128];
            snprintf(path, sizeof path, "/sys/class/kfd/kfd/proc/%ld/vram_%u", pid, gpu_id);
            if (FILE* f = fopen(path, "r")) {
                unsigned long long v = 0;
                if (fscanf(f, "%llu", &v) == 1) out.emplace_back(pid, (uint64_t)v);
                fclose(f);
            }
        }
        closedir(d);
    }
    std::sort(out.begin(), out.end());
    return out;
}

// This process's pid in KFD's accounting.  The directory names are pids of the host's pid namespace, which a
// process in a container does not know (getpid() differs), so it is found by a probe: the one process whose
// vram_<gpu_id> grows by exactly a 64 MiB device allocation made in between two reads.  Probed lazily, by the
// first co-tenant check (a twin launch that could add companions, or the counter), never at tv_create; a probe that
// finds no single match (another allocation in this process or another one at the same moment) is retried on a later
// check, at most once a second.  Only the process that created the ctx probes: in a forked child (getpid() differs
// from c->create_pid) no HIP call is made and there is no check.  0 = not known (no check: companions stay on).
static long kfd_self_pid(tv_ctx* c) {
    static std::mutex mu;
    static long self = 0, for_pid = -1;
    static std::chrono::steady_clock::time_point failed_at;
    static bool failed = false;
    const long me = (long)getpid();
    if (me != c->create_pid) return 0;
    std::lock_guard<std::mutex> g(mu);
    if (for_pid == me && self) return self;
    const auto now = std::chrono::steady_clock::now();
    if (for_pid == me && failed && now - failed_at < std::chrono::seconds(1)) return 0;
    for_pid = me;
    self = 0;
    constexpr uint64_t kProbe = 64ull << 20;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(c->device) != hipSuccess) {
        (void)hipGetLastError();
        failed = true;
        failed_at = now;
        return 0;
    }
    for (int attempt = 0; attempt < 3 && !self; attempt++) {
        const auto before = kfd_vram(c->kfd_gpu_id);
        void* p = nullptr;
        if (hipMalloc(&p, kProbe) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        const auto after = kfd_vram(c->kfd_gpu_id);
        (void)hipFree(p);
        long found = 0;
        int matches = 0;
        for (const auto& [pid, v] : after) {
            auto it = std::lower_bound(before.begin(), before.end(), std::make_pair(pid, (uint64_t)0));
            const uint64_t was = (it != before.end() && it->first == pid) ? it->second : 0;
            if (v == was + kProbe) {
                found = pid;
                matches++;
            }
        }
        if (matches == 1) self = found;   // another process allocating exactly 64 MiB at the same time: again
    }
    (void)hipSetDevice(prev);
    failed = self == 0;
    failed_at = now;
    return self;
}

// The KFD gpu_id of HIP device `device` for the co-tenant check: the topology node whose PCI location matches
// (0 = none; no HIP allocation is made here: the process's own entry is found later, kfd_self_pid).
uint32_t kfd_gpu_id(int device) { return kfd_topology_gpu_id(device); }

// The gpu_id when the co-tenant check can run (the GPU is in the topology and this process's entry in the
// accounting is known, probing for it now if need be), else 0.
uint32_t kfd_check_id(tv_ctx* c) { return (c->kfd_gpu_id && kfd_self_pid(c)) ? c->kfd_gpu_id : 0; }

// Bytes of this GPU's memory other processes hold (KFD's per-process accounting,
// /sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>), or 0 when it cannot be read.  Cached for a second.
uint64_t cotenant_vram(tv_ctx* c) {
    if (!c->kfd_gpu_id) return 0;
    const auto now = std::chrono::steady_clock::now();
    if (c->cotenant_checked && now - c->cotenant_at < std::chrono::seconds(1)) return c->cotenant_bytes;
    const long self = kfd_self_pid(c);
    uint64_t sum = 0;
    if (self)
        for (const auto& [pid, v] : kfd_vram(c->kfd_gpu_id))
            if (pid != self) sum += v;
    c->cotenant_bytes = sum;
    c->cotenant_at = now;
    c->cotenant_checked = self != 0;   // (an unresolved probe is retried by the next check, not cached)
    return sum;
}

bool companions_on(tv_ctx* c) {
    if (c->twin_fill == 0) return false;
    if (c->twin_fill >= 2) return true;
    return cotenant_vram(c) < kCotenantBytes;   // auto: not on a GPU another process is using
}

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


uint64_t piece_len(const tv_ctx* c, uint64_t i) {  // piece.ts:16-19
    if (i == c->P - 1 && c->total % c->L) return c->total % c->L;
    return c->L;
}

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


// The CPUs the context's library threads run on: the GPU's NUMA node when bound, else none (unpinned).

void apply_numa(tv_ctx* c) {
    for (auto& p : c->pool) p.set_affinity(numa_cpus(c), c->proc_cpus_ok ? &c->proc_cpus : nullptr);
}

int ensure_ring(tv_ctx* c, int which) {
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
int take_slot(tv_ctx* c, int* slot, int which) {
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
int release_slot(tv_ctx* c, int slot, int which) {
    RingRef r = ring_ref(c, which);
    r.lent[slot] = false;
    TV_HIP(c, hipEventRecord(r.ev[slot], lane_stream(c, which)));
    return TV_OK;
}

// A lent slot that goes back to the ring on every exit of its scope (error paths included).

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
    const bool unhashed = c->win && c->any_unhashed;
    if (!avail_bits && !c->any_file_bad && !unhashed) {
        *out = c->d_base_avail;
        return TV_OK;
    }
    TV_HIP(c, hipEventSynchronize(c->ev_avail));  // the previous copy out of h_avail is done
    const size_t nbytes = c->bit_words * 8, used = (c->count + 7) / 8;
    for (size_t k = 0; k < nbytes; k++) {
        const uint8_t caller = k < used ? (avail_bits ? avail_bits[k] : 0xFF) : 0;
        const uint8_t bad = k < used ? (uint8_t)(c->file_bad[k] | (unhashed ? c->unhashed[k] : 0)) : 0;
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
int launch_resident(tv_ctx* c, const TvPieces& p_in, int kernel, bool hash, hipStream_t on, bool alone) {
    TvPieces p = p_in;
    p.lane_pairs = lane_pairs_for(c, p.n);
    if (!alone) {
        // a window's hash beside others on the hash streams: its real grid only (companions would fill every CU and
        // keep the windows hashing beside it from their CUs)
        TV_HIP(c, tv_launch_verify(p, kernel, hash, on ? on : c->stream, c->split_pairs, &c->last_workgroups));
        return TV_OK;
    }
    // A CU running ONE 2-wave twin workgroup spends ~80 more shader cycles per block than one running two
    // (PMC GRBM_GUI_ACTIVE: 1,806 vs 1,727; sleeping fillers do not help, working ones do: DESIGN.md section 5).
    // With fewer real workgroups than 2 per CU, companions fill the grid to 2 x CUs: they re-hash main
    // workgroups' pieces on otherwise idle SIMDs and discard the result (TV_OPT_TWIN_FILL, default on).
    if (kernel == TV_KERNEL_TWIN && !c->twin_pack && (c->split_pairs < 2 || c->split_pairs > 5) && companions_on(c)) {
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
        std::lock_guard<std::mutex> g(c->slot_mu);  // (a tv_stage_files helper may stage on lane 1 meanwhile)
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
    if (c->slots) {
        std::lock_guard<std::mutex> g(c->slot_mu);  // (as piece_dst: a lane-1 helper may take a slot meanwhile)
        if (!c->slot_of.count(i - c->first))
            return fail(c, TV_ERR_STATE, "piece %llu holds no slot (it was never staged, or was listed since)",
                        (unsigned long long)i);
    }
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
    for (uint64_t j = j0; j < j1; j++) set_bit(c->unhashed.data(), j);  // (never staged: never verified)
    c->any_unhashed = true;
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

// The stream window w's hash runs on: the compute stream, then the layout's extra hash streams in turn.  (HIP maps
// streams onto GPU_MAX_HW_QUEUES hardware queues, 4 by default; a hash queued behind another stream's wait on the
// same hardware queue waits with it, so the hashes use the compute stream and hash streams created next to it, and
// nothing else waits on the compute stream during a pass: fills of windows go on the staging lane.)
hipStream_t win_hash_stream(const tv_ctx* c, uint64_t seq) {
    const uint64_t k = seq % (uint64_t)std::max(1, c->win_nhs);
    return k == 0 ? c->stream : c->win_hs[k - 1];
}

// Hash the open window (no-op when none is open): on its hash stream, after every copy and fill queued into its
// buffer on either staging lane.
int win_seal(tv_ctx* c) {
    if (c->win_cur == UINT64_MAX) return TV_OK;
    const uint64_t j0 = c->win_cur * c->win_n, n = std::min(c->win_n, c->count - j0);
    hipStream_t hs = win_hash_stream(c, c->win_launched);
    for (int l = 0; l < 2; l++) {
        TV_HIP(c, hipEventRecord(c->win_cp[l], lane_stream(c, l)));
        TV_HIP(c, hipStreamWaitEvent(hs, c->win_cp[l], 0));
    }
    if (c->win_launched == 0) TV_HIP(c, hipEventRecord(c->ev_k0, hs));
    const TvPieces p = window_launch(c, j0, n, win_base(c, c->win_buf));
    const int kernel = choose_kernel_n(c, n, p.n_main < p.n);
    const int rc = launch_resident(c, p, kernel, /*hash=*/true, hs, /*alone=*/c->win_nhs <= 1);
    if (rc) return rc;
    TV_HIP(c, hipEventRecord(c->win_ev[c->win_buf], hs));
    c->last_kernel = kernel;
    c->win_launched++;
    c->win_valid = j0 + n;
    c->win_cur = UINT64_MAX;
    return TV_OK;
}

// Everything queued on the hash streams, joined into the compute stream (the compare, digest reads and zeroing
// after a pass follow every window's hash).
int win_join(tv_ctx* c) {
    for (int k = 0; k + 1 < c->win_nhs; k++) {
        TV_HIP(c, hipEventRecord(c->win_hs_ev[k], c->win_hs[k]));
        TV_HIP(c, hipStreamWaitEvent(c->stream, c->win_hs_ev[k], 0));
    }
    return TV_OK;
}

// Wait for every hash stream (before the payload is freed or re-planned, and at tv_destroy).
int win_sync_streams(tv_ctx* c) {
    for (int k = 0; k < kWinHashStreams - 1; k++)
        if (c->win_hs[k]) TV_HIP(c, hipStreamSynchronize(c->win_hs[k]));
    return TV_OK;
}

// Open window w for staging.  A window of this pass already hashed is TV_ERR_STATE: staging ascends.
int win_enter(tv_ctx* c, uint64_t w) {
    if (c->win_done) {  // the last pass was finalized: this stage starts a new one
        c->win_done = false;
        c->win_valid = 0;
        c->win_launched = 0;
        c->win_timing = false;
        std::fill(c->unhashed.begin(), c->unhashed.end(), 0);
        c->any_unhashed = false;
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
    // the buffer is free once the kernel that last read it is done (copies and fills on either lane wait for it)
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
    if (!rc) rc = win_join(c);
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

// Linear byte where window w's pieces end (the next window's first byte; the shard's end for the last one).
uint64_t win_end_linear(const tv_ctx* c, uint64_t w) {
    const uint64_t j1 = std::min(c->count, (w + 1) * c->win_n);
    const uint64_t last = c->first + j1 - 1;
    return last * c->L + piece_len(c, last);
}

// The state every non-stream call needs.  need_resident: the call reads or writes the resident payload
// (absent with TV_OPT_RESIDENT = 0).  Calls sharing the output / chunk buffers wait for a stream to end.
int require_layout(tv_ctx* c, bool need_digests, bool need_resident) {
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
int dma_h2d(tv_ctx* c, uint8_t* dst, const uint8_t* src, uint64_t n, int lane) {
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
int stage_copy(tv_ctx* c, uint64_t pos, const uint8_t* src, uint64_t n, bool pinned, int lane,
               bool src_in_ring) {
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
                int lane, bool src_in_ring) {
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

}  // namespace tvi
