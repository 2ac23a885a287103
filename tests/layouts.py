"""Seeded synthetic torrent layouts for parity tests (regenerated identically on the GPU box).

Payload bytes: linear offset o -> byte (o & 7) of splitmix64(seed, o >> 3) (the generator
oracle/sha1_oracle.c and the device fill kernel implement; its definition is pinned in
tests/test_oracle.py).  Digests are hashlib SHA-1 of the CLEAN payload; corruption then flips
one bit inside each chosen piece.  `missing` files are absent on disk and `short` files are
truncated, so pieces touching their bytes are unreadable (Storage.get -> null, storage.ts:50-65).

Config 1 of BASELINE.json is the layout "cfg1" (64 MiB single file, 256 KiB pieces, 256 pieces;
three corrupted, including piece 0 and the final piece).
Config 3 of BASELINE.json is the layout "cfg3": 10,000 files of U[0, 524288] bytes (>= 20
zero-length, >= 5 under 64 B), 256 KiB pieces, short final piece, 1 % corrupted pieces
including piece 0, the final piece and >= 10 pieces that span a file boundary.
"""
from __future__ import annotations

import bisect
import hashlib
import random

from torrent_amd.metainfo import FileInfo, make_info

LAYOUTS = [
    {"name": "single_short_last", "seed": 101, "piece_length": 65536, "sizes": [5_000_001],
     "corrupt_frac": 0.02},
    {"name": "multi_zero_tiny", "seed": 102, "piece_length": 16384, "n_files": 300, "max_size": 40000,
     "zero": 20, "tiny": 5, "corrupt_frac": 0.01},
    {"name": "many_tiny_span", "seed": 103, "piece_length": 1024, "n_files": 1000, "max_size": 100,
     "zero": 50, "tiny": 200, "corrupt_frac": 0.05},
    {"name": "missing_and_short", "seed": 104, "piece_length": 32768, "n_files": 50, "max_size": 200000,
     "zero": 3, "tiny": 2, "corrupt_frac": 0.03, "missing": [7, 31], "short": {12: 1000, 40: 0}},
    {"name": "exact_multiple", "seed": 105, "piece_length": 4096, "sizes": [4096 * 33, 4096 * 7],
     "corrupt_frac": 0.0},
    # BASELINE config 1 (the reference's CPU-runnable case): one 64 MiB file, 256 KiB pieces, 256 pieces
    {"name": "cfg1", "seed": 1, "piece_length": 262144, "sizes": [64 << 20], "corrupt_frac": 0.01},
    {"name": "cfg3", "seed": 3, "piece_length": 262144, "n_files": 10000, "max_size": 524288,
     "zero": 20, "tiny": 5, "corrupt_frac": 0.01, "span_corrupt": 10, "big": True},
]


def by_name(name: str) -> dict:
    for s in LAYOUTS:
        if s["name"] == name:
            return s
    raise KeyError(name)


def _sizes(spec: dict, rng: random.Random):
    if "sizes" in spec:
        return list(spec["sizes"])
    n = spec["n_files"]
    sizes = [rng.randrange(spec["max_size"] + 1) for _ in range(n)]
    idx = rng.sample(range(n), spec.get("zero", 0) + spec.get("tiny", 0))
    for k in idx[:spec.get("zero", 0)]:
        sizes[k] = 0
    for k in idx[spec.get("zero", 0):]:
        sizes[k] = rng.randrange(1, 64)
    return sizes


def build_layout(spec: dict, fill=None) -> dict:
    """fill(seed, off, n): the byte generator -- the oracle's by default (tests); tools and bench.py pass
    tests/synth.py's numpy restatement of it (pinned equal in test_oracle.py), so they call nothing under oracle/."""
    if fill is None:
        from oracle import oracle as O  # the byte generator only (pinned in test_oracle.py)
        fill = O.synth_fill

    rng = random.Random(spec["seed"])
    sizes = _sizes(spec, rng)
    L = spec["piece_length"]
    total = sum(sizes)
    files = [FileInfo(length=s, path=[f"d{k % 7}", f"f{k:05d}.bin"]) for k, s in enumerate(sizes)]
    clean = fill(spec["seed"], 0, total)
    P = -(-total // L)
    pieces_raw = b"".join(hashlib.sha1(bytes(clean[i * L:min(total, (i + 1) * L)])).digest()
                          for i in range(P))
    payload = clean  # corrupted in place below
    starts = [0]
    for s in sizes:
        starts.append(starts[-1] + s)

    def plen(i):
        return (total % L) if (i == P - 1 and total % L) else L

    # corruption: piece 0, the final piece, spanning pieces, random pieces up to the fraction
    corrupted = set()
    n_bad = int(round(spec["corrupt_frac"] * P))
    if n_bad:
        corrupted |= {0, P - 1}
        if spec.get("span_corrupt"):
            spanning = [i for i in range(P)
                        if bisect.bisect_right(starts, i * L) != bisect.bisect_left(starts, i * L + plen(i))]
            corrupted |= set(rng.sample(spanning, spec["span_corrupt"]))
        while len(corrupted) < max(n_bad, len(corrupted)):
            corrupted.add(rng.randrange(P))
    for i in sorted(corrupted):
        o = i * L + rng.randrange(plen(i))
        payload[o] ^= 1 << rng.randrange(8)

    # on-disk availability
    missing = set(spec.get("missing", []))
    short = dict(spec.get("short", {}))
    have = [0 if k in missing else min(sizes[k], short.get(k, sizes[k])) for k in range(len(sizes))]

    def readable(lo, hi):
        """Bytes [lo, hi) all present on disk (zero-length reads always succeed)."""
        if hi <= lo:
            return True
        k = bisect.bisect_right(starts, lo) - 1
        while k < len(sizes) and starts[k] < hi:
            a, b = max(lo, starts[k]), min(hi, starts[k + 1])
            if b > a and (b - starts[k]) > have[k]:
                return False
            k += 1
        return True

    def read_piece(i):
        lo, n = i * L, plen(i)
        if lo + n > total or not readable(lo, lo + n):
            return None
        return bytes(payload[lo:lo + n])

    single = not ("n_files" in spec or len(sizes) > 1)

    def disk_files():
        """{path tuple: on-disk bytes} for a MemoryStorage (missing files absent).  A single-file
        torrent's file is [name] (storage.ts:99-101)."""
        out = {}
        if single:
            return {} if 0 in missing else {(spec["name"],): bytes(payload[:have[0]])}
        for k, f in enumerate(files):
            if k in missing:
                continue
            out[tuple(f.path)] = bytes(payload[starts[k]:starts[k] + have[k]])
        return out

    avail = bytearray((P + 7) // 8)
    for i in range(P):
        if readable(i * L, i * L + plen(i)):
            avail[i >> 3] |= 0x80 >> (i & 7)

    info = make_info(L, pieces_raw, spec["name"], files=None if single else files,
                     length=total)
    return {"info": info, "payload": payload, "pieces": [pieces_raw[20 * i:20 * i + 20] for i in range(P)],
            "pieces_raw": pieces_raw, "n_pieces": P, "total_length": total, "corrupted": sorted(corrupted),
            "read_piece": read_piece, "disk_files": disk_files, "avail": bytes(avail), "sizes": sizes,
            "starts": starts}
