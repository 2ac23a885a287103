/*
 * oracle/sha1_oracle.c -- CPU restatement of the reference's piece-verification path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker.  The product
 * path (torrent_amd/, libtorrent_verify.so) never links or calls it.
 *
 * Parity status: PINNED.  The reference's SHA-1 path is WebCrypto
 * `crypto.subtle.digest("SHA-1", content)` (reference tools/make_torrent.ts:28-31;
 * also metainfo.ts:141-143).  That code lives in the Deno runtime (Rust `ring`,
 * software SHA-1), which is absent here, so it is restated from FIPS 180-4.
 * The restatement is pinned by the reference's own fixtures:
 * test_data/singlefile.torrent (1706 digests) and test_data/multifile.torrent
 * (1855 digests) were produced by make_torrent.ts.  Their payloads are
 * reconstructible ("0\n" x 447,135,744 B; plus "7\n" x 525,148,160 B), and
 * tests/test_oracle.py checks every one of the 3,561 digests.
 *
 * Layout rules restated here (each function cites the reference line it follows):
 *   piece length ............ piece.ts:16-19
 *   piece -> linear offset ... torrent.ts:165,186
 *   digest unpacking ......... metainfo.ts:111 + _bytes.ts:92-99 (a short final slice never matches)
 *   have-bitfield bit order .. torrent.ts:53,60 and :147-149 (MSB-first, spare bits 0)
 *
 * Synthetic payloads (bench / GPU tests) use a counter PRNG so that the GPU box
 * regenerates them: byte at linear offset o = byte (o & 7), little-endian, of
 * splitmix64(seed, o >> 3).  The device fill kernel implements the same function.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))

/* FIPS 180-4 section 6.1.2: one 512-bit block.  Fully unrolled, 16-word rolling schedule
 * (the usual scalar formulation; ring's software SHA-1 is the same class of code). */
#define ORC_BLK(i) (w[(i) & 15] = ORC_ROTL(w[((i) + 13) & 15] ^ w[((i) + 8) & 15] ^ w[((i) + 2) & 15] ^ w[(i) & 15], 1))
#define ORC_R0(v, x, y, z, u, i) u += ((x & (y ^ z)) ^ z) + w[i] + 0x5A827999u + ORC_ROTL(v, 5); x = ORC_ROTL(x, 30);
#define ORC_R1(v, x, y, z, u, i) u += ((x & (y ^ z)) ^ z) + ORC_BLK(i) + 0x5A827999u + ORC_ROTL(v, 5); x = ORC_ROTL(x, 30);
#define ORC_R2(v, x, y, z, u, i) u += (x ^ y ^ z) + ORC_BLK(i) + 0x6ED9EBA1u + ORC_ROTL(v, 5); x = ORC_ROTL(x, 30);
#define ORC_R3(v, x, y, z, u, i) u += (((x | y) & z) | (x & y)) + ORC_BLK(i) + 0x8F1BBCDCu + ORC_ROTL(v, 5); x = ORC_ROTL(x, 30);
#define ORC_R4(v, x, y, z, u, i) u += (x ^ y ^ z) + ORC_BLK(i) + 0xCA62C1D6u + ORC_ROTL(v, 5); x = ORC_ROTL(x, 30);
#define ORC_5(R, i) R(a, b, c, d, e, (i)) R(e, a, b, c, d, (i) + 1) R(d, e, a, b, c, (i) + 2) \
                    R(c, d, e, a, b, (i) + 3) R(b, c, d, e, a, (i) + 4)
static void orc_compress(uint32_t h[5], const uint8_t *blk) {
    uint32_t w[16];
    for (int t = 0; t < 16; t++)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
               ((uint32_t)blk[4 * t + 2] << 8) | (uint32_t)blk[4 * t + 3];
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    ORC_5(ORC_R0, 0) ORC_5(ORC_R0, 5) ORC_5(ORC_R0, 10)
    ORC_R0(a, b, c, d, e, 15) ORC_R1(e, a, b, c, d, 16) ORC_R1(d, e, a, b, c, 17)
    ORC_R1(c, d, e, a, b, 18) ORC_R1(b, c, d, e, a, 19)
    ORC_5(ORC_R2, 20) ORC_5(ORC_R2, 25) ORC_5(ORC_R2, 30) ORC_5(ORC_R2, 35)
    ORC_5(ORC_R3, 40) ORC_5(ORC_R3, 45) ORC_5(ORC_R3, 50) ORC_5(ORC_R3, 55)
    ORC_5(ORC_R4, 60) ORC_5(ORC_R4, 65) ORC_5(ORC_R4, 70) ORC_5(ORC_R4, 75)
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

/* Same compression with the x86 SHA extensions (SHA-NI): sha1rnds4 runs 4 rounds, sha1nexte
 * derives the next E (rotl30 of the old A) plus 4 message words, and sha1msg1/2 expand the
 * schedule W[t] = rotl1(W[t-3]^W[t-8]^W[t-14]^W[t-16]).  It is the CPU baseline's fast path: the
 * reference's own SHA-1 (WebCrypto in the Deno runtime) is native code of this class, and the
 * SURVEY (sec. 8d) asks for the baseline at that speed, not a slow scalar port.  The scalar
 * orc_compress above stays as the plain FIPS restatement; tests check both. */
#if defined(__x86_64__)
#include <immintrin.h>
#define ORC_NI_GROUP(g, f)                                                                          \
    do {                                                                                            \
        __m128i mg;                                                                                 \
        if ((g) < 4)                                                                                \
            mg = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blk + 16 * (g))), rev);        \
        else                                                                                        \
            mg = _mm_sha1msg2_epu32(_mm_xor_si128(_mm_sha1msg1_epu32(m[((g) - 4) & 3], m[((g) - 3) & 3]), \
                                                  m[((g) - 2) & 3]),                                \
                                    m[((g) - 1) & 3]);                                              \
        m[(g) & 3] = mg;                                                                            \
        __m128i ev = (g) == 0 ? _mm_add_epi32(e0, mg) : _mm_sha1nexte_epu32(prev, mg);              \
        prev = abcd;                                                                                \
        abcd = _mm_sha1rnds4_epu32(abcd, ev, f);                                                    \
    } while (0)
__attribute__((target("sha,ssse3,sse4.1"))) static void orc_compress_ni(uint32_t h[5], const uint8_t *blk,
                                                                         size_t nblocks) {
    const __m128i rev = _mm_set_epi64x(0x0001020304050607ll, 0x08090a0b0c0d0e0fll);
    __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)h), 0x1B);
    __m128i e0 = _mm_set_epi32((int)h[4], 0, 0, 0);
    for (; nblocks; nblocks--, blk += 64) {
        const __m128i abcd0 = abcd, e00 = e0;
        __m128i m[4], prev = abcd;
        ORC_NI_GROUP(0, 0); ORC_NI_GROUP(1, 0); ORC_NI_GROUP(2, 0); ORC_NI_GROUP(3, 0); ORC_NI_GROUP(4, 0);
        ORC_NI_GROUP(5, 1); ORC_NI_GROUP(6, 1); ORC_NI_GROUP(7, 1); ORC_NI_GROUP(8, 1); ORC_NI_GROUP(9, 1);
        ORC_NI_GROUP(10, 2); ORC_NI_GROUP(11, 2); ORC_NI_GROUP(12, 2); ORC_NI_GROUP(13, 2); ORC_NI_GROUP(14, 2);
        ORC_NI_GROUP(15, 3); ORC_NI_GROUP(16, 3); ORC_NI_GROUP(17, 3); ORC_NI_GROUP(18, 3); ORC_NI_GROUP(19, 3);
        e0 = _mm_sha1nexte_epu32(prev, e00);
        abcd = _mm_add_epi32(abcd, abcd0);
    }
    _mm_storeu_si128((__m128i *)h, _mm_shuffle_epi32(abcd, 0x1B));
    h[4] = (uint32_t)_mm_extract_epi32(e0, 3);
}
#endif

static void orc_compress_scalar(uint32_t h[5], const uint8_t *blk, size_t nblocks) {
    for (; nblocks; nblocks--, blk += 64) orc_compress(h, blk);
}

/* 1 = scalar FIPS restatement, 2 = SHA-NI.  Default: the fastest the host supports. */
static void (*orc_blocks)(uint32_t *, const uint8_t *, size_t) = 0;
static int orc_impl_id = 0;

static int orc_have_ni(void) {
#if defined(__x86_64__)
    __builtin_cpu_init();
    return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
#else
    return 0;
#endif
}

/* Select the compression: 0 = best available, 1 = scalar, 2 = SHA-NI.  Returns the selected
 * implementation, or -1 if the request is unsupported on this host (selection unchanged). */
int orc_set_impl(int impl) {
    if (impl == 0) impl = orc_have_ni() ? 2 : 1;
    if (impl == 2 && !orc_have_ni()) return -1;
    if (impl != 1 && impl != 2) return -1;
#if defined(__x86_64__)
    orc_blocks = impl == 2 ? orc_compress_ni : orc_compress_scalar;
#else
    orc_blocks = orc_compress_scalar;
#endif
    orc_impl_id = impl;
    return impl;
}
int orc_get_impl(void) {
    if (!orc_blocks) orc_set_impl(0);
    return orc_impl_id;
}

/* Incremental interface (FIPS 180-4 5.1.1 padding). */
typedef struct { uint32_t h[5]; uint64_t n; uint8_t buf[64]; uint32_t fill; } orc_sha1_ctx;

static void orc_init(orc_sha1_ctx *c) {
    if (!orc_blocks) orc_set_impl(0);
    c->h[0] = 0x67452301u; c->h[1] = 0xEFCDAB89u; c->h[2] = 0x98BADCFEu;
    c->h[3] = 0x10325476u; c->h[4] = 0xC3D2E1F0u; c->n = 0; c->fill = 0;
}
static void orc_update(orc_sha1_ctx *c, const uint8_t *p, uint64_t len) {
    c->n += len;
    if (c->fill) {
        while (len && c->fill < 64) { c->buf[c->fill++] = *p++; len--; }
        if (c->fill == 64) { orc_blocks(c->h, c->buf, 1); c->fill = 0; }
    }
    if (len >= 64) {
        size_t nb = (size_t)(len / 64);
        orc_blocks(c->h, p, nb);
        p += 64 * (uint64_t)nb; len -= 64 * (uint64_t)nb;
    }
    while (len) { c->buf[c->fill++] = *p++; len--; }
}
static void orc_final(orc_sha1_ctx *c, uint8_t out[20]) {
    uint64_t bits = c->n * 8;
    uint8_t pad = 0x80;
    orc_update(c, &pad, 1);
    uint8_t z = 0;
    while (c->fill != 56) orc_update(c, &z, 1);
    uint8_t lenb[8];
    for (int i = 0; i < 8; i++) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
    orc_update(c, lenb, 8);
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)(c->h[i] >> 24); out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 8); out[4 * i + 3] = (uint8_t)c->h[i];
    }
}

/* SHA-1 of one byte string: the restatement of crypto.subtle.digest("SHA-1", content),
 * make_torrent.ts:29. */
void orc_sha1(const uint8_t *data, uint64_t len, uint8_t out[20]) {
    orc_sha1_ctx c; orc_init(&c); orc_update(&c, data, len); orc_final(&c, out);
}

/* piece.ts:16-19: (n === info.pieces.length - 1 && info.length % info.pieceLength) || info.pieceLength
 * n_pieces is the DIGEST COUNT (info.pieces.length), not ceil(length / pieceLength). */
uint64_t orc_piece_len(uint64_t n, uint64_t n_pieces, uint64_t total_length, uint64_t piece_length) {
    if (n == n_pieces - 1 && (total_length % piece_length) != 0) return total_length % piece_length;
    return piece_length;
}

/* Number of digest slices partition(info.pieces, 20) yields (_bytes.ts:92-99): ceil(len/20). */
uint64_t orc_n_pieces(uint64_t pieces_bytes) { return (pieces_bytes + 19) / 20; }

static inline void orc_set_bit(uint8_t *bf, uint64_t i) { bf[i >> 3] |= (uint8_t)(0x80u >> (i & 7)); } /* torrent.ts:147-149 */
static inline int orc_get_bit(const uint8_t *bf, uint64_t i) { return (bf[i >> 3] >> (7 - (i & 7))) & 1; }

/*
 * Verify every piece of a linear payload (the concatenation of the torrent's files in
 * info.files order, storage.ts:89-137) against info.pieces.
 *   piece i: offset i*L (torrent.ts:165), length orc_piece_len (piece.ts:16-19);
 *   unreadable (offset+len > total, or avail bit clear) => bit 0 (Storage.get -> null);
 *   digest slice shorter than 20 B (pieces_bytes % 20 != 0) => never equal => bit 0;
 *   bitfield_out: ceil(P/8) bytes, MSB-first, spare bits 0 (torrent.ts:53,60,147-149).
 * avail may be NULL (= all readable).  Returns P.
 */
uint64_t orc_verify_linear(const uint8_t *payload, uint64_t total_length, uint64_t piece_length,
                           const uint8_t *pieces, uint64_t pieces_bytes, const uint8_t *avail,
                           uint8_t *bitfield_out) {
    uint64_t P = orc_n_pieces(pieces_bytes);
    memset(bitfield_out, 0, (P + 7) / 8);
    for (uint64_t i = 0; i < P; i++) {
        uint64_t off = i * piece_length, len = orc_piece_len(i, P, total_length, piece_length);
        if (off + len > total_length) continue;
        if (avail && !orc_get_bit(avail, i)) continue;
        if (20 * i + 20 > pieces_bytes) continue;
        uint8_t d[20];
        orc_sha1(payload + off, len, d);
        if (memcmp(d, pieces + 20 * i, 20) == 0) orc_set_bit(bitfield_out, i);
    }
    return P;
}

/* ---- synthetic payloads ------------------------------------------------------------ */

static inline uint64_t orc_splitmix64(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* out[j] = synthetic byte at linear offset off + j. */
void orc_synth_fill(uint64_t seed, uint64_t off, uint64_t len, uint8_t *out) {
    uint64_t j = 0;
    while (j < len && ((off + j) & 7)) {
        uint64_t o = off + j;
        out[j++] = (uint8_t)(orc_splitmix64(seed, o >> 3) >> (8 * (o & 7)));
    }
    for (; j + 8 <= len; j += 8) {
        uint64_t v = orc_splitmix64(seed, (off + j) >> 3);
        memcpy(out + j, &v, 8); /* little-endian host */
    }
    for (; j < len; j++) {
        uint64_t o = off + j;
        out[j] = (uint8_t)(orc_splitmix64(seed, o >> 3) >> (8 * (o & 7)));
    }
}

/* ---- threaded drivers (CPU baseline / ground truth) -------------------------------- */

typedef struct {
    int mode; /* 0: hash synthetic pieces, 1: hash pieces of a linear buffer */
    uint64_t seed; const uint8_t *payload;
    uint64_t total, L, P, first, count;
    uint8_t *out;
    uint64_t next; pthread_mutex_t mu;
} orc_job;

static void *orc_worker(void *arg) {
    orc_job *j = (orc_job *)arg;
    uint8_t *buf = NULL; uint64_t cap = 0;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint64_t k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->count) break;
        uint64_t i = j->first + k;
        uint64_t off = i * j->L, len = orc_piece_len(i, j->P, j->total, j->L);
        if (off + len > j->total) { memset(j->out + 20 * k, 0, 20); continue; }
        if (j->mode == 0) {
            /* stream the synthetic bytes through a 64 KiB window: no full-piece buffer */
            if (!buf) { cap = 65536; buf = (uint8_t *)malloc(cap); }
            orc_sha1_ctx c; orc_init(&c);
            for (uint64_t p = 0; p < len; p += cap) {
                uint64_t n = len - p < cap ? len - p : cap;
                orc_synth_fill(j->seed, off + p, n, buf);
                orc_update(&c, buf, n);
            }
            orc_final(&c, j->out + 20 * k);
        } else {
            orc_sha1(j->payload + off, len, j->out + 20 * k);
        }
    }
    free(buf);
    return NULL;
}

static void orc_run(orc_job *j, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    pthread_mutex_init(&j->mu, NULL);
    j->next = 0;
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, orc_worker, j);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j->mu);
}

/* SHA-1 digests (20 B each) of synthetic pieces [first, first+count) of a torrent with
 * total_length bytes, piece_length L and n_pieces digests. */
void orc_synth_piece_digests(uint64_t seed, uint64_t total_length, uint64_t piece_length,
                             uint64_t n_pieces, uint64_t first, uint64_t count, int threads,
                             uint8_t *out) {
    orc_job j;
    memset(&j, 0, sizeof j);
    j.mode = 0; j.seed = seed; j.total = total_length; j.L = piece_length; j.P = n_pieces;
    j.first = first; j.count = count; j.out = out;
    orc_run(&j, threads);
}

/* SHA-1 digests of pieces [first, first+count) of a linear payload buffer (creation mode,
 * make_torrent.ts:147-173 for single files, :62-113 for files concatenated in order). */
void orc_hash_pieces(const uint8_t *payload, uint64_t total_length, uint64_t piece_length,
                     uint64_t n_pieces, uint64_t first, uint64_t count, int threads, uint8_t *out) {
    orc_job j;
    memset(&j, 0, sizeof j);
    j.mode = 1; j.payload = payload; j.total = total_length; j.L = piece_length; j.P = n_pieces;
    j.first = first; j.count = count; j.out = out;
    orc_run(&j, threads);
}
