// tv_host.cpp -- host-only helpers of libtorrent_verify.so (see tv_host.h).
#include "tv_host.h"

#include <string.h>

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

inline uint8_t byte_at(uint64_t seed, uint64_t o) { return (uint8_t)(splitmix64(seed, o >> 3) >> (8 * (o & 7))); }

}  // namespace

void tv_synth_fill_host(uint64_t seed, uint64_t off, uint64_t n, uint8_t* out) {
    uint64_t j = 0;
    for (; j < n && ((off + j) & 7); j++) out[j] = byte_at(seed, off + j);
    const uint64_t nw = (n - j) / 8;
#if defined(__x86_64__)
    if (have_avx512()) words_avx512(seed, (off + j) >> 3, nw, out + j);
    else
#endif
        words_portable(seed, (off + j) >> 3, nw, out + j);
    for (j += 8 * nw; j < n; j++) out[j] = byte_at(seed, off + j);
}
