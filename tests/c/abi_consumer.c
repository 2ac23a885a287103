/*
 * tests/c/abi_consumer.c -- a plain-C consumer of libtorrent_verify.so, with no Python and no
 * torch: the shape of what a Deno FFI / cgo / JNI binding does ("the build's C++
 * test/bench drivers ... must exercise the identical ABI because Deno is absent here").
 *
 *   abi_consumer cpu   checks the version, the no-device and NULL-argument error paths, and the
 *                      error messages (runs anywhere)
 *   abi_consumer gpu   checks the full path on device 0 with the reference's own conventions:
 *                      pieces "abc" | "def" | "g" (L = 3, short last piece, piece.ts:16-19), the
 *                      middle digest corrupted, MSB-first bitfield (torrent.ts:147-149) = 0xA0.
 *                      It covers verify, hash, verify_list, verify_host from pageable and pinned
 *                      memory, read-back, stage_file (incl. short / missing files -> TV_ERR_IO),
 *                      and two contexts driven from two threads at once.
 *
 * Build: gcc -O2 -Iinclude tests/c/abi_consumer.c -Ltorrent_amd -ltorrent_verify \
 *            -Wl,-rpath,$PWD/torrent_amd -lpthread -o abi_consumer
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "torrent_verify.h"

static int failures = 0;
#define CHECK(cond, ...)                                                     \
    do {                                                                     \
        if (!(cond)) {                                                       \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);            \
            fprintf(stderr, __VA_ARGS__);                                    \
            fprintf(stderr, "\n");                                           \
            failures++;                                                      \
        }                                                                    \
    } while (0)
#define OK(call, ctx)                                                        \
    do {                                                                     \
        int rc_ = (call);                                                    \
        if (rc_ != TV_OK) {                                                  \
            char m_[512];                                                    \
            tv_last_error((ctx), m_, sizeof m_);                             \
            fprintf(stderr, "FAIL %s:%d: %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_, m_); \
            failures++;                                                      \
        }                                                                    \
    } while (0)

static const char *PAYLOAD = "abcdefg";
static const char *HEX[3] = {"a9993e364706816aba3e25717850c26c9cd0d89d",  /* sha1("abc") */
                             "589c22335a381f122d129225f5c0ba3056ed5811",  /* sha1("def") */
                             "54fd1711209fb1c0781092374132c66e79e2241b"}; /* sha1("g")   */

static void unhex(const char *h, uint8_t *out) {
    for (int i = 0; i < 20; i++) {
        unsigned v;
        sscanf(h + 2 * i, "%2x", &v);
        out[i] = (uint8_t)v;
    }
}

static int run_cpu(void) {
    CHECK(tv_abi_version() == TV_ABI_VERSION, "abi version %d", tv_abi_version());
    int n = -1;
    CHECK(tv_device_count(&n) == TV_OK && n >= 0, "device count");
    CHECK(tv_device_count(NULL) == TV_ERR_ARG, "NULL count must be TV_ERR_ARG");
    char msg[256];
    CHECK(tv_last_error(NULL, msg, sizeof msg) > 0 && strlen(msg) > 0, "thread error message");
    CHECK(tv_set_layout(NULL, 7, 3, 3, 0, 3) == TV_ERR_ARG, "NULL ctx");
    CHECK(tv_verify(NULL, NULL, NULL) == TV_ERR_ARG, "NULL ctx verify");
    CHECK(tv_host_alloc(16, NULL) == TV_ERR_ARG, "NULL out");
    uint32_t cores = 0;
    CHECK(tv_cpu_share(&cores) == TV_OK && cores >= 1, "cpu share %u", cores);
    CHECK(tv_cpu_share(NULL) == TV_ERR_ARG, "NULL cores must be TV_ERR_ARG");
    {
        const uint64_t lens[1] = {7};
        int32_t st[1];
        CHECK(tv_stage_file_table(NULL, 1, lens, "a", 2, st) == TV_ERR_ARG, "NULL ctx file table");
        uint8_t bf[1];
        CHECK(tv_stream_file_table(NULL, 1, lens, "a", 2, NULL, bf, st) == TV_ERR_ARG, "NULL ctx streamed file table");
    }
    if (n == 0) {  /* no GPU: creating a context is an error with a message, never a crash */
        tv_ctx *c = NULL;
        int rc = tv_create(&c, 0);
        CHECK(rc < 0 && c == NULL, "tv_create without a device must fail (rc %d)", rc);
        CHECK(tv_last_error(NULL, msg, sizeof msg) > 0, "message after tv_create failure");
    }
    return failures;
}

struct shard_job { int device; uint64_t first, count; const uint8_t *digests; uint8_t out[8]; int rc; };

static void *verify_shard(void *arg) {
    struct shard_job *j = (struct shard_job *)arg;
    tv_ctx *c = NULL;
    j->rc = tv_create(&c, j->device);
    if (j->rc) return NULL;
    /* 40 pieces of 3 bytes (a synthetic "abc" torrent): 120 bytes */
    uint8_t payload[120];
    for (int i = 0; i < 120; i++) payload[i] = (uint8_t)("abc"[i % 3]);
    if (!(j->rc = tv_set_layout(c, 120, 3, 40, j->first, j->count)) &&
        !(j->rc = tv_set_digests(c, j->digests, 40 * 20)) && !(j->rc = tv_stage(c, 0, payload, 120)))
        j->rc = tv_verify(c, NULL, j->out);
    tv_destroy(c);
    return NULL;
}

static int run_gpu(void) {
    int n = 0;
    OK(tv_device_count(&n), NULL);
    CHECK(n > 0, "no GPU visible");
    if (n == 0) return failures + 1;
    uint8_t digests[60];
    for (int i = 0; i < 3; i++) unhex(HEX[i], digests + 20 * i);
    uint8_t good[60];
    memcpy(good, digests, 60);
    digests[20 + 7] ^= 0x01; /* corrupt piece 1's digest */

    tv_ctx *c = NULL;
    OK(tv_create(&c, 0), NULL);
    OK(tv_set_layout(c, 7, 3, 3, 0, 3), c);
    OK(tv_set_digests(c, digests, 60), c);
    OK(tv_stage(c, 0, (const uint8_t *)PAYLOAD, 7), c);
    uint8_t bf = 0xFF;
    OK(tv_verify(c, NULL, &bf), c);
    CHECK(bf == 0xA0, "bitfield %02x, want a0", bf);

    uint8_t avail = 0x80; /* only piece 0 readable */
    OK(tv_verify(c, &avail, &bf), c);
    CHECK(bf == 0x80, "bitfield with avail %02x, want 80", bf);

    uint8_t dig[60];
    OK(tv_hash(c, dig), c);
    CHECK(memcmp(dig, good, 60) == 0, "tv_hash digests differ from sha1(abc|def|g)");

    uint64_t list[3] = {2, 1, 0};
    uint8_t ok[3] = {9, 9, 9};
    OK(tv_verify_list(c, list, 3, ok), c);
    CHECK(ok[0] == 1 && ok[1] == 0 && ok[2] == 1, "verify_list %d%d%d, want 101", ok[0], ok[1], ok[2]);

    char back[8] = {0};
    OK(tv_read(c, 0, (uint8_t *)back, 7), c);
    CHECK(memcmp(back, PAYLOAD, 7) == 0, "tv_read returned %.7s", back);

    /* streamed from pageable, then from pinned host memory */
    OK(tv_verify_host(c, (const uint8_t *)PAYLOAD, 7, NULL, &bf), c);
    CHECK(bf == 0xA0, "verify_host bitfield %02x", bf);
    void *pinned = NULL;
    OK(tv_host_alloc(7, &pinned), NULL);
    if (pinned) {
        memcpy(pinned, PAYLOAD, 7);
        OK(tv_verify_host(c, (const uint8_t *)pinned, 7, NULL, &bf), c);
        CHECK(bf == 0xA0, "verify_host (pinned) bitfield %02x", bf);
        OK(tv_host_free(pinned), NULL);
    }
    char msg0[256];
    /* from a file: "xx" + payload at file offset 2 (fsStorage.get's open/seek/read, storage.ts:150-172) */
    char path[] = "/tmp/tv_abi_consumer_XXXXXX";
    int fd = mkstemp(path);
    CHECK(fd >= 0, "mkstemp");
    if (fd >= 0) {
        CHECK(write(fd, "xxabcdefg", 9) == 9, "write");
        close(fd);
        OK(tv_set_layout(c, 7, 3, 3, 0, 3), c);
        OK(tv_set_digests(c, digests, 60), c);
        OK(tv_stage_file(c, path, 2, 0, 7), c);
        OK(tv_verify(c, NULL, &bf), c);
        CHECK(bf == 0xA0, "stage_file bitfield %02x, want a0", bf);
        CHECK(tv_stage_file(c, path, 5, 0, 7) == TV_ERR_IO, "short file must be TV_ERR_IO");
        CHECK(tv_last_error(c, msg0, sizeof msg0) > 0 && strstr(msg0, "bytes"), "message: %s", msg0);
        CHECK(tv_stage_file(c, "/nonexistent/tv_file", 0, 0, 7) == TV_ERR_IO, "missing file must be TV_ERR_IO");
        /* zero-length segments still open the path as fsStorage.get does (storage.ts:109-110,158) */
        CHECK(tv_stage_file(c, "/nonexistent/tv_file", 0, 0, 0) == TV_ERR_IO, "zero-length, missing parent dir");
        CHECK(tv_stage_file(c, "/tmp", 0, 0, 0) == TV_ERR_IO, "zero-length on a directory must be TV_ERR_IO");
        char absent[] = "/tmp/tv_abi_consumer_absent_XXXXXX";
        int afd = mkstemp(absent);
        if (afd >= 0) { close(afd); unlink(absent); }
        OK(tv_stage_file(c, absent, 0, 0, 0), c); /* a missing file in a writable directory opens */
        CHECK(access(absent, F_OK) != 0, "tv_stage_file must not create %s", absent);
        /* one tv_stage_files call: the data segment, then zero-length segments on piece 2 (a directory),
           piece 1 (a missing directory) and piece 0 (a missing file in /tmp: fine, not created) */
        {
            /* a fresh layout: the failed calls above marked pieces 0-2 unreadable until the next one */
            OK(tv_set_layout(c, 7, 3, 3, 0, 3), c);
            OK(tv_set_digests(c, digests, 60), c);
            const char *paths[4] = {path, "/tmp", "/nonexistent/tv_file", absent};
            const uint64_t fo[4] = {2, 0, 0, 0}, lin[4] = {0, 6, 3, 0}, lens[4] = {7, 0, 0, 0};
            int32_t st[4] = {9, 9, 9, 9};
            OK(tv_stage_files(c, 4, paths, fo, lin, lens, st), c);
            CHECK(st[0] == TV_OK && st[1] == TV_ERR_IO && st[2] == TV_ERR_IO && st[3] == TV_OK,
                  "stage_files statuses %d %d %d %d", st[0], st[1], st[2], st[3]);
            CHECK(access(absent, F_OK) != 0, "tv_stage_files must not create %s", absent);
            /* the library marks piece lin / L of each failed zero-length segment itself */
            OK(tv_verify(c, NULL, &bf), c);
            CHECK(bf == 0x80, "stage_files zero-length bitfield %02x, want 80", bf);
            /* a short file: its whole pieces before the end are staged and stay readable, the rest are
               marked unreadable by the library (Storage.get reads piece by piece, storage.ts:50-65) */
            CHECK(truncate(path, 7) == 0, "truncate");  /* "xxabcde": 5 of the segment's 7 bytes */
            const uint64_t lin1[1] = {0}, lens1[1] = {7}, fo1[1] = {2};
            const char *p1[1] = {path};
            OK(tv_set_layout(c, 7, 3, 3, 0, 3), c);
            OK(tv_set_digests(c, digests, 60), c);
            OK(tv_stage(c, 0, (const uint8_t *)"zzzdefg", 7), c); /* piece 0 wrong, pieces 1-2 right */
            OK(tv_stage_files(c, 1, p1, fo1, lin1, lens1, st), c);
            CHECK(st[0] == TV_ERR_IO, "short segment status %d", st[0]);
            OK(tv_verify(c, NULL, &bf), c);
            CHECK(bf == 0x80, "short segment bitfield %02x, want 80", bf);
        }
        unlink(path);
    }

    double kms = -1, tms = -1;
    OK(tv_last_timing(c, &kms, &tms), c);
    CHECK(kms >= 0 && tms >= kms, "timings %f %f", kms, tms);

    /* errors come back as status + message, never a crash */
    CHECK(tv_set_layout(c, 60, 3, 20, 3, 1) == TV_ERR_ARG, "shard_first %% 8 != 0 must be TV_ERR_ARG");
    char msg[256];
    CHECK(tv_last_error(c, msg, sizeof msg) > 0 && strstr(msg, "multiple of 8"), "message: %s", msg);
    tv_destroy(c);

    /* two contexts on two host threads at once (one GPU here): shards [0,24) and [24,40) */
    uint8_t d40[800];
    uint8_t abc[20];
    unhex(HEX[0], abc);
    for (int i = 0; i < 40; i++) memcpy(d40 + 20 * i, abc, 20);
    d40[20 * 5] ^= 1;
    d40[20 * 31] ^= 1;
    struct shard_job jobs[2] = {{0, 0, 24, d40, {0}, 0}, {0, 24, 16, d40, {0}, 0}};
    pthread_t th[2];
    for (int t = 0; t < 2; t++) pthread_create(&th[t], NULL, verify_shard, &jobs[t]);
    for (int t = 0; t < 2; t++) pthread_join(th[t], NULL);
    CHECK(jobs[0].rc == 0 && jobs[1].rc == 0, "threaded shards rc %d %d", jobs[0].rc, jobs[1].rc);
    uint8_t all[5];
    memcpy(all, jobs[0].out, 3);
    memcpy(all + 3, jobs[1].out, 2);
    const uint8_t want[5] = {0xFB, 0xFF, 0xFF, 0xFE, 0xFF}; /* pieces 5 and 31 bad */
    CHECK(memcmp(all, want, 5) == 0, "threaded bitfield %02x %02x %02x %02x %02x", all[0], all[1], all[2],
          all[3], all[4]);
    return failures;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "cpu";
    int f = strcmp(mode, "gpu") == 0 ? run_gpu() : run_cpu();
    printf("%s: %s (%d failures)\n", mode, f ? "FAILED" : "ok", f);
    return f ? 1 : 0;
}
