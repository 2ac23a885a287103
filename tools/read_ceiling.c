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
 * shared buffer of that size at (t mod (bytes / part)) * part, as the library's readers fill its ring slots.
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
static uint64_t* task_file;   /* task -> file; offset = (task - first task of the file) * part */
static uint64_t* first_task;
static atomic_uint_fast64_t next_task, total_bytes;
static int direct;

static int (*host_alloc)(uint64_t, void**);
static char* spread_buf;
static uint64_t spread_parts;
static cpu_set_t node_cpus;
static int pin_node;

static void* worker(void* arg) {
    (void)arg;
    if (pin_node) sched_setaffinity(0, sizeof node_cpus, &node_cpus);
    char* buf = NULL;
    if (host_alloc) {
        void* p = NULL;
        if (host_alloc(part, &p) == 0) buf = p;
    }
    const int own = buf == NULL;
    if (own) buf = aligned_alloc(4096, part);
    for (;;) {
        const uint64_t t = atomic_fetch_add(&next_task, 1);
        if (t >= ntasks) break;
        file_t* f = &files[task_file[t]];
        uint64_t off = (t - first_task[task_file[t]]) * part, n = f->size - off < part ? f->size - off : part;
        while (n) {
            const uint64_t ask = direct ? (n + 4095) / 4096 * 4096 : n;
            char* dst = spread_buf ? spread_buf + (t % spread_parts) * part : buf;
            const ssize_t got = pread(f->fd, dst, ask, (off_t)off);
            if (got <= 0) break;
            const uint64_t g = (uint64_t)got < n ? (uint64_t)got : n;
            atomic_fetch_add(&total_bytes, g);
            off += g;
            n -= g;
            if ((uint64_t)got < ask && n) break;
        }
    }
    if (own) free(buf);   /* (a tv_host_alloc buffer lives until the process ends) */
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int threads = atoi(argv[1]);
    part = strtoull(argv[2], NULL, 10);
    direct = argc > 3 && strcmp(argv[3], "direct") == 0;
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
        ntasks += (files[k].size + part - 1) / part;
    }
    task_file = malloc((ntasks + 1) * sizeof(uint64_t));
    for (uint64_t k = 0; k < nfiles; k++)
        for (uint64_t t = first_task[k]; t < first_task[k] + (files[k].size + part - 1) / part; t++) task_file[t] = k;
    pthread_t* th = malloc(threads * sizeof(pthread_t));
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, worker, NULL);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    const uint64_t b = atomic_load(&total_bytes);
    printf("{\"bytes\": %llu, \"seconds\": %.4f, \"gbps\": %.3f, \"files\": %llu, \"threads\": %d, \"part\": %llu, "
           "\"direct\": %d}\n", (unsigned long long)b, s, (double)b / s / 1e9, (unsigned long long)nfiles, threads,
           (unsigned long long)part, direct);
    return 0;
}
