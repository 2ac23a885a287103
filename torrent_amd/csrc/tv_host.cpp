// tv_host.cpp -- host-only helpers of libtorrent_verify.so (see tv_host.h).
#include "tv_host.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace {

inline uint64_t splitmix64(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Whole 8-byte words w0 .. w0 + nw - 1 to o (any alignment).  The same loop twice: the AVX-512 clone
// vectorises the three 64-bit multiplies (vpmullq), the portable one cannot.
#if defined(__x86_64__)
__attribute__((target("avx512f,avx512dq,avx512vl"))) void words_avx512(uint64_t seed, uint64_t w0, uint64_t nw,
                                                                        uint8_t* o) {
    for (uint64_t k = 0; k < nw; k++) {
        const uint64_t v = splitmix64(seed, w0 + k);
        memcpy(o + 8 * k, &v, 8);
    }
}
#endif

// Large fills (the streamed resume check's producer writing 64 MiB pinned ring slots that only the DMA engine
// reads): eight splitmix64 words per AVX-512 vector, written with non-temporal stores.  A plain store first
// reads the line (read for ownership), so the producer would move 2 bytes over the memory bus per byte
// produced, in competition with the DMA engine reading the slots it filled earlier.
__attribute__((target("avx512f,avx512dq,avx512vl"))) void words_avx512_nt(uint64_t seed, uint64_t w0, uint64_t nw,
                                                                           uint8_t* o) {
    uint64_t k = 0;
    for (; k < nw && ((uintptr_t)(o + 8 * k) & 63); k++) {
        const uint64_t v = splitmix64(seed, w0 + k);
        memcpy(o + 8 * k, &v, 8);
    }
    const __m512i lane = _mm512_set_epi64(7, 6, 5, 4, 3, 2, 1, 0);
    const __m512i vseed = _mm512_set1_epi64((long long)seed);
    const __m512i c0 = _mm512_set1_epi64((long long)0x9E3779B97F4A7C15ull);
    const __m512i c1 = _mm512_set1_epi64((long long)0xBF58476D1CE4E5B9ull);
    const __m512i c2 = _mm512_set1_epi64((long long)0x94D049BB133111EBull);
    for (; k + 8 <= nw; k += 8) {
        const __m512i i1 = _mm512_add_epi64(_mm512_set1_epi64((long long)(w0 + k + 1)), lane);  // index + 1
        __m512i z = _mm512_add_epi64(vseed, _mm512_mullo_epi64(i1, c0));
        z = _mm512_mullo_epi64(_mm512_xor_si512(z, _mm512_srli_epi64(z, 30)), c1);
        z = _mm512_mullo_epi64(_mm512_xor_si512(z, _mm512_srli_epi64(z, 27)), c2);
        z = _mm512_xor_si512(z, _mm512_srli_epi64(z, 31));
        _mm512_stream_si512(reinterpret_cast<__m512i*>(o + 8 * k), z);
    }
    for (; k < nw; k++) {
        const uint64_t v = splitmix64(seed, w0 + k);
        memcpy(o + 8 * k, &v, 8);
    }
    _mm_sfence();   // the non-temporal stores are globally visible before the caller hands the slot to DMA
}

void words_portable(uint64_t seed, uint64_t w0, uint64_t nw, uint8_t* o) {
    for (uint64_t k = 0; k < nw; k++) {
        const uint64_t v = splitmix64(seed, w0 + k);
        memcpy(o + 8 * k, &v, 8);
    }
}

bool have_avx512() {
#if defined(__x86_64__)
    static const bool yes = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
               __builtin_cpu_supports("avx512vl");
    }();
    return yes;
#else
    return false;
#endif
}

bool nt_enabled();

inline uint8_t byte_at(uint64_t seed, uint64_t o) { return (uint8_t)(splitmix64(seed, o >> 3) >> (8 * (o & 7))); }

}  // namespace

void tv_synth_fill_host(uint64_t seed, uint64_t off, uint64_t n, uint8_t* out) {
    uint64_t j = 0;
    for (; j < n && ((off + j) & 7); j++) out[j] = byte_at(seed, off + j);
    const uint64_t nw = (n - j) / 8;
#if defined(__x86_64__)
    if (have_avx512() && nw >= 8192 && nt_enabled()) words_avx512_nt(seed, (off + j) >> 3, nw, out + j);   // >= 64 KiB
    else if (have_avx512()) words_avx512(seed, (off + j) >> 3, nw, out + j);
    else
#endif
        words_portable(seed, (off + j) >> 3, nw, out + j);
    for (j += 8 * nw; j < n; j++) out[j] = byte_at(seed, off + j);
}

namespace {

bool nt_enabled() {
    static const bool on = [] {
        const char* e = getenv("TORRENT_VERIFY_NT_STORES");
        return !(e && e[0] == '0');
    }();
    return on;
}

#if defined(__x86_64__)
__attribute__((target("avx512f"))) void copy_avx512_nt(uint8_t* dst, const uint8_t* src, uint64_t n) {
    const uint64_t head = std::min<uint64_t>(n, (64 - ((uintptr_t)dst & 63)) & 63);
    memcpy(dst, src, head);
    uint64_t k = head;
    for (; k + 256 <= n; k += 256) {
        const __m512i a = _mm512_loadu_si512(src + k), b = _mm512_loadu_si512(src + k + 64);
        const __m512i c = _mm512_loadu_si512(src + k + 128), d = _mm512_loadu_si512(src + k + 192);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + k), a);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + k + 64), b);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + k + 128), c);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + k + 192), d);
    }
    for (; k + 64 <= n; k += 64) _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + k), _mm512_loadu_si512(src + k));
    memcpy(dst + k, src + k, n - k);
    _mm_sfence();
}
#endif

}  // namespace

void tv_copy_host(uint8_t* dst, const uint8_t* src, uint64_t n) {
#if defined(__x86_64__)
    if (n >= (64u << 10) && have_avx512() && nt_enabled()) {
        copy_avx512_nt(dst, src, n);
        return;
    }
#endif
    memcpy(dst, src, n);
}
