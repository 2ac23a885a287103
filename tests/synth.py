"""The synthetic payload generator in numpy, and piece digests with hashlib: input generation and checking for the
tools and bench.py without calling anything under oracle/ (test infrastructure the product and its measurement
tools do not run).

fill(seed, off, n): byte (o & 7) of splitmix64(seed, o >> 3) for linear offsets o in [off, off + n) -- the
generator oracle/sha1_oracle.c (orc_synth_fill) and the device fill kernel (tv_fill_words_kernel) implement;
tests/test_oracle.py::test_numpy_generator_equals_the_oracles pins the three together.
"""
from __future__ import annotations

import hashlib
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_CHUNK_WORDS = 1 << 21          # 16 MiB of payload per numpy pass (bounded temporaries)


def _words(seed: int, w0: int, nw: int) -> np.ndarray:
    """splitmix64(seed, w) for w in [w0, w0 + nw), as little-endian uint64 words."""
    z = np.arange(w0 + 1, w0 + nw + 1, dtype=np.uint64)
    z *= _GAMMA                                 # (uint64 arithmetic wraps, as the C does)
    z += np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    z ^= z >> np.uint64(30)
    z *= _M1
    z ^= z >> np.uint64(27)
    z *= _M2
    z ^= z >> np.uint64(31)
    return z.astype("<u8", copy=False)


def fill_into(out, seed: int, off: int, threads: int = 0) -> None:
    """Write the generator's bytes for [off, off + len(out)) into the writable buffer `out`."""
    mv = memoryview(out).cast("B")
    n = mv.nbytes
    if n == 0:
        return
    dst = np.frombuffer(mv, dtype=np.uint8)
    w_first, w_end = off >> 3, (off + n + 7) >> 3
    spans = [(w, min(w_end, w + _CHUNK_WORDS)) for w in range(w_first, w_end, _CHUNK_WORDS)]

    def one(span):
        a, b = span
        raw = _words(seed, a, b - a).view(np.uint8)
        lo = max(off, a * 8)                    # linear bytes [lo, hi) of this span inside the request
        hi = min(off + n, b * 8)
        dst[lo - off:hi - off] = raw[lo - a * 8:hi - a * 8]

    threads = threads or min(16, os.cpu_count() or 1)
    if threads <= 1 or len(spans) == 1:
        for s in spans:
            one(s)
    else:
        with ThreadPoolExecutor(threads) as ex:   # (numpy releases the GIL in its ufuncs)
            list(ex.map(one, spans))


def fill(seed: int, off: int, n: int, threads: int = 0) -> bytearray:
    out = bytearray(n)
    fill_into(out, seed, off, threads)
    return out


def piece_digests(seed: int, total: int, L: int, P: int, threads: int = 0) -> bytes:
    """hashlib SHA-1 of every piece of the generator's payload of `total` bytes (pieces of L; the last one short)."""
    def one(i):
        lo = i * L
        return hashlib.sha1(fill(seed, lo, min(L, total - lo), threads=1)).digest()

    threads = threads or min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(threads) as ex:       # (hashlib releases the GIL on large buffers)
        return b"".join(ex.map(one, range(P)))


def hash_pieces(buf, L: int, P: int, threads: int = 0) -> bytes:
    """hashlib SHA-1 of the pieces of `buf` (pieces of L; the last one short)."""
    mv = memoryview(buf).cast("B")
    total = mv.nbytes

    def one(i):
        return hashlib.sha1(mv[i * L:min(total, (i + 1) * L)]).digest()

    threads = threads or min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(threads) as ex:
        return b"".join(ex.map(one, range(P)))
