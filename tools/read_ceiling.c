/* read_ceiling.c -- what the box's storage delivers: every file named on stdin (one path per line) read with
 * pread in `part`-byte requests by `threads` threads taking (file, offset) tasks from a shared counter, bytes
 * dropped.  Prints {"bytes": B, "seconds": S, "gbps": G}.  The storage benches (tools/storage_paths_bench.py) run it
 * after dropping the files from the page cache, so the cold legs have a ceiling measured without Python in the
 * way (the round-4 Python reader under-measured it for 10,000 small files).
 * A third argument "direct" opens the files O_DIRECT (reads bypass the page cache; the length of each request is
 * rounded up to 4 KiB, the file end returns short).
 * Environment (probes of what the library's reader differs in): RC_HOST_ALLOC_LIB=<libtorrent_verify.so> reads into
 * buffers from its tv_host_alloc (page-locked, as the library's staging ring); RC_CPU_NODE=<n> pins the readers to the
 * CPUs of NUMA node n (as the library pins its readers next to the GPU); RC_SPREAD=<bytes> reads request t into a
 * shared buffer of that size at (t mod (bytes / part)) * part, as the library's readers fill its ring slots;
 * RC_BOUNCE=copy reads every request into the reader's own reused buffer and then memcpy's it to its RC_SPREAD place
 * (does a compact read destination plus a host copy keep the reused-buffer rate?); RC_BOUNCE=dma gives each reader two
 * reused page-locked buffers (hipHostMalloc) and its own HIP stream, and DMAs every request from them to a 1 GiB device
 * buffer (hipMemcpyAsync at (t mod 256) * part), the next read into a buffer waiting for the DMA that last read it
 * (compact destination, no host copy: the library's cold path without its 192 MiB ring); RC_BOUNCE=dma1 the same with
 * ONE stream shared by every reader (the library's form: the bounce DMAs queued on the staging lane's copy stream).
 * RC_STRIDE=<bytes> (a multiple of the part) orders the requests column-major, as the library's streamed columns read
 * a file: part c of every stride-long piece before part c + 1 of any (is the disk's rate for such reads the bound of
 * a cold streamed verify?).
 * build: gcc -O2 -pthread tools/read_ceiling.c -o read_ceiling -ldl;  usage: read_ceiling THREADS PART_BYTES [direct] < paths */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

typedef struct { char* path; uint64_t size; int fd; } file_t;
static file_t* files;
static uint64_t nfiles, part, ntasks;
static uint64_t stride;   /* RC_STRIDE: column-major tasks (see the header comment); 0 = sequential parts */
static uint64_t* task_file;   /* task -> file; offset = (task - first task of the file) * part */
static uint64_t* first_task;
static atomic_uint_fast64_t next_task, total_bytes;
static int direct;

static int (*host_alloc)(uint64_t, void**);
static char* spread_buf;
static uint64_t spread_parts;
static cpu_set_t node_cpus;
static int pin_node;

/* RC_BOUNCE (libamdhip64 entry points, looked up at run time so the tool still builds with gcc alone) */
static int bounce;   /* 0 off, 1 copy, 2 dma */
static void* shared_stream;   /* RC_BOUNCE=dma1 */
typedef int (*hip_i_t)(int);
typedef int (*hip_malloc_t)(void**, size_t);
typedef int (*hip_host_malloc_t)(void**, size_t, unsigned);
typedef int (*hip_stream_create_t)(void**);
typedef int (*hip_memcpy_async_t)(void*, const void*, size_t, int, void*);
typedef int (*hip_event_create_t)(void**, unsigned);
typedef int (*hip_event_record_t)(void*, void*);
typedef int (*hip_event_sync_t)(void*);
typedef int (*hip_stream_sync_t)(void*);
static hip_i_t hip_set_device;
static hip_malloc_t hip_malloc;
static hip_host_malloc_t hip_host_malloc;
static hip_stream_create_t hip_stream_create;
static hip_memcpy_async_t hip_memcpy_async;
static hip_event_create_t hip_event_create;
static hip_event_record_t hip_event_record;
static hip_event_sync_t hip_event_sync;
static hip_stream_sync_t hip_stream_sync;
static char* dev_buf;
static const uint64_t dev_parts = 256;
static atomic_int hip_errors;

static void* worker(void* arg) {
    (void)arg;
    if (pin_node) sched_setaffinity(0, sizeof node_cpus, &node_cpus);
    char* buf = NULL;
    char* dbuf[2] = {NULL, NULL};   /* RC_BOUNCE=dma: two page-locked buffers, each with the event of its last DMA */
    void* dev[2] = {NULL, NULL};
    void* stream = NULL;
    int k = 0;
    if (bounce == 2) {
        hip_set_device(0);
        for (int i = 0; i < 2; i++) {
            if (hip_host_malloc((void**)&dbuf[i], part, 0) || hip_event_create(&dev[i], 2)) atomic_fetch_add(&hip_errors, 1);
        }
        if (shared_stream) stream = shared_stream;
        else if (hip_stream_create(&stream)) atomic_fetch_add(&hip_errors, 1);
        if (atomic_load(&hip_errors)) return NULL;
    } else if (host_alloc) {
        void* p = NULL;
        if (host_alloc(part, &p) == 0) buf = p;
    }
    const int own = buf == NULL && bounce != 2;
    if (own) buf = aligned_alloc(4096, part);
    int recorded[2] = {0, 0};
    for (;;) {
        const uint64_t t = atomic_fetch_add(&next_task, 1);
        if (t >= ntasks) break;
        file_t* f = &files[task_file[t]];
        uint64_t off = (t - first_task[task_file[t]]) * part;
        if (stride) {   /* column-major: every piece's part `col` before any piece's part col + 1 */
            const uint64_t i = t - first_task[task_file[t]], np = (f->size + stride - 1) / stride;
            off = (i % np) * stride + (i / np) * part;
            if (off >= f->size) continue;
        }
        uint64_t n = f->size - off < part ? f->size - off : part;
        char* into = buf;
        if (bounce == 2) {   /* the buffer's last DMA must be done before it is read into again */
            if (recorded[k] && hip_event_sync(dev[k])) atomic_fetch_add(&hip_errors, 1);
            into = dbuf[k];
        } else if (spread_buf && bounce == 0) {
            into = spread_buf + (t % spread_parts) * part;
        }
        uint64_t done = 0;
        while (n) {
            const uint64_t ask = direct ? (n + 4095) / 4096 * 4096 : n;
            const ssize_t got = pread(f->fd, into + done, ask, (off_t)off);
            if (got <= 0) break;
            const uint64_t g = (uint64_t)got < n ? (uint64_t)got : n;
            atomic_fetch_add(&total_bytes, g);
            off += g;
            n -= g;
            done += g;
            if ((uint64_t)got < ask && n) break;
        }
        if (bounce == 1 && spread_buf && done) memcpy(spread_buf + (t % spread_parts) * part, into, done);
        if (bounce == 2 && done) {
            if (hip_memcpy_async(dev_buf + (t % dev_parts) * part, into, done, 1 /* host to device */, stream) ||
                hip_event_record(dev[k], stream))
                atomic_fetch_add(&hip_errors, 1);
            recorded[k] = 1;
            k ^= 1;
        }
    }
    if (bounce == 2 && stream && hip_stream_sync(stream)) atomic_fetch_add(&hip_errors, 1);
    if (own) free(buf);   /* (a tv_host_alloc / hipHostMalloc buffer lives until the process ends) */
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int threads = atoi(argv[1]);
    part = strtoull(argv[2], NULL, 10);
    direct = argc > 3 && strcmp(argv[3], "direct") == 0;
    if (getenv("RC_STRIDE")) {
        stride = strtoull(getenv("RC_STRIDE"), NULL, 10);
        if (stride && (stride % part || stride < part)) return 2;   /* a whole number of parts per stride */
    }
    const char* lib = getenv("RC_HOST_ALLOC_LIB");
    if (lib && lib[0]) {
        void* h = dlopen(lib, RTLD_NOW);
        if (h) host_alloc = (int (*)(uint64_t, void**))dlsym(h, "tv_host_alloc");
        if (!host_alloc) { fprintf(stderr, "RC_HOST_ALLOC_LIB: %s\n", dlerror()); return 3; }
    }
    const char* spread = getenv("RC_SPREAD");
    if (spread && spread[0]) {
        const uint64_t sb = strtoull(spread, NULL, 10) / part * part;
        spread_parts = sb / part;
        if (spread_parts) {
            void* p = NULL;
            if (host_alloc && host_alloc(sb, &p) == 0) spread_buf = p;
            else spread_buf = aligned_alloc(4096, sb);
            memset(spread_buf, 0, sb);
        }
    }
    const char* bn = getenv("RC_BOUNCE");
    if (bn && bn[0]) {
        bounce = strncmp(bn, "dma", 3) == 0 ? 2 : 1;
        if (bounce == 2) {
            void* h = dlopen("libamdhip64.so", RTLD_NOW);
            if (!h) { fprintf(stderr, "RC_BOUNCE=dma: %s\n", dlerror()); return 3; }
            hip_set_device = (hip_i_t)dlsym(h, "hipSetDevice");
            hip_malloc = (hip_malloc_t)dlsym(h, "hipMalloc");
            hip_host_malloc = (hip_host_malloc_t)dlsym(h, "hipHostMalloc");
            hip_stream_create = (hip_stream_create_t)dlsym(h, "hipStreamCreate");
            hip_memcpy_async = (hip_memcpy_async_t)dlsym(h, "hipMemcpyAsync");
            hip_event_create = (hip_event_create_t)dlsym(h, "hipEventCreateWithFlags");
            hip_event_record = (hip_event_record_t)dlsym(h, "hipEventRecord");
            hip_event_sync = (hip_event_sync_t)dlsym(h, "hipEventSynchronize");
            hip_stream_sync = (hip_stream_sync_t)dlsym(h, "hipStreamSynchronize");
            if (!hip_set_device || !hip_malloc || !hip_host_malloc || !hip_stream_create || !hip_memcpy_async ||
                !hip_event_create || !hip_event_record || !hip_event_sync || !hip_stream_sync) {
                fprintf(stderr, "RC_BOUNCE=dma: a HIP entry point is missing\n");
                return 3;
            }
            if (hip_set_device(0) || hip_malloc((void**)&dev_buf, dev_parts * part)) {
                fprintf(stderr, "RC_BOUNCE=dma: hipMalloc failed\n");
                return 3;
            }
            if (strcmp(bn, "dma1") == 0 && hip_stream_create(&shared_stream)) {
                fprintf(stderr, "RC_BOUNCE=dma1: hipStreamCreate failed\n");
                return 3;
            }
        }
    }
    const char* node = getenv("RC_CPU_NODE");
    if (node && node[0]) {
        char path[128], list[4096];
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", atoi(node));
        FILE* f = fopen(path, "r");
        if (f && fgets(list, sizeof list, f)) {
            CPU_ZERO(&node_cpus);
            for (char* tok = strtok(list, ",\n"); tok; tok = strtok(NULL, ",\n")) {
                int a = 0, b = 0;
                if (sscanf(tok, "%d-%d", &a, &b) == 2) { for (int c = a; c <= b; c++) CPU_SET(c, &node_cpus); }
                else if (sscanf(tok, "%d", &a) == 1) CPU_SET(a, &node_cpus);
            }
            cpu_set_t mine;
            if (sched_getaffinity(0, sizeof mine, &mine) == 0) CPU_AND(&node_cpus, &node_cpus, &mine);
            pin_node = CPU_COUNT(&node_cpus) > 0;
        }
        if (f) fclose(f);
    }
    uint64_t cap = 1024;
    files = malloc(cap * sizeof(file_t));
    char line[8192];
    while (fgets(line, sizeof line, stdin)) {
        line[strcspn(line, "\n")] = 0;
        if (!line[0]) continue;
        if (nfiles == cap) files = realloc(files, (cap *= 2) * sizeof(file_t));
        files[nfiles].path = strdup(line);
        nfiles++;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);   /* the opens are part of reading the files */
    first_task = malloc((nfiles + 1) * sizeof(uint64_t));
    for (uint64_t k = 0; k < nfiles; k++) {
        struct stat st;
        files[k].fd = open(files[k].path, O_RDONLY | (direct ? O_DIRECT : 0));
        files[k].size = (files[k].fd >= 0 && fstat(files[k].fd, &st) == 0) ? (uint64_t)st.st_size : 0;
        first_task[k] = ntasks;
        ntasks += stride ? (files[k].size + stride - 1) / stride * (stride / part) : (files[k].size + part - 1) / part;
    }
    first_task[nfiles] = ntasks;
    task_file = malloc((ntasks + 1) * sizeof(uint64_t));
    for (uint64_t k = 0; k < nfiles; k++)
        for (uint64_t t = first_task[k]; t < first_task[k + 1]; t++) task_file[t] = k;
    pthread_t* th = malloc(threads * sizeof(pthread_t));
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, worker, NULL);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    const uint64_t b = atomic_load(&total_bytes);
    printf("{\"bytes\": %llu, \"seconds\": %.4f, \"gbps\": %.3f, \"files\": %llu, \"threads\": %d, \"part\": %llu, "
           "\"direct\": %d, \"bounce\": %d, \"hip_errors\": %d}\n", (unsigned long long)b, s, (double)b / s / 1e9,
           (unsigned long long)nfiles, threads, (unsigned long long)part, direct, bounce, atomic_load(&hip_errors));
    return atomic_load(&hip_errors) ? 4 : 0;
}
