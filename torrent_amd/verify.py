"""Piece verification on MI355X -- the host-side mirror of the new `verify.ts` module.

The reference (rclarey/torrent) has no verify function.  This module adds it
by composing the reference's own pieces, exactly as SURVEY.md 3(D) states:

    for i < P = info.pieces.length (metainfo.ts:16):
        off_i = i * pieceLength                                   (torrent.ts:165)
        len_i = pieceLength(i, info)                              (piece.ts:16-19)
        bytes = storage.get(off_i, len_i)   # null => bit 0       (storage.ts:50-65)
        bit i = SHA-1(bytes) == info.pieces[i]                    (make_torrent.ts:28-31)
    bitfield: ceil(P/8) bytes, byte i>>3 |= 0x80 >> (i % 8)       (torrent.ts:53,60,147-149)

The SHA-1 work runs in libtorrent_verify.so (HIP, gfx950): the bytes are staged into HBM and
one kernel verifies every piece (one lane per piece).  There is no CPU fallback: without the
library or a GPU these functions raise.

Public API (names follow the reference's camelCase surface, snake_cased):
    verify_pieces(info, storage, devices=None) -> bytearray         (verifyPieces)
    verify_piece(info, index, data) -> bool                         (verifyPiece)
    verify_payload(info, payload, devices=None, resident=True) -> bytearray
    hash_pieces(payload, piece_length, devices=None) -> bytes       (creation mode, make_torrent.ts)
and asyncio wrappers verify_pieces_async / verify_piece_async (the reference API is Promise-based).
"""
from __future__ import annotations

import asyncio
import threading
from concurrent.futures import ThreadPoolExecutor
from contextlib import contextmanager
from typing import List, Optional, Sequence

from . import _native
from .metainfo import InfoDict
from .piece import piece_length

# pieces gathered per tv_stage call when reading through a Storage
_STAGE_BATCH_BYTES = 256 << 20
# verify_files: file segments at least this long are DMA'd from the page cache (tv_stage_file)
_DIRECT_MIN_BYTES = 32 << 20


def shard_ranges(n_pieces: int, n_shards: int) -> List[tuple]:
    """Contiguous piece ranges, each starting at a multiple of 8 pieces so every shard's
    bitfield slice is whole bytes.  Returns [(first, count), ...]."""
    n_shards = max(1, n_shards)
    per = -(-n_pieces // n_shards)
    per = -(-per // 8) * 8
    out = []
    first = 0
    for _ in range(n_shards):
        count = max(0, min(per, n_pieces - first))
        out.append((first, count))
        first += count
    return out


def _set_bit(bf: bytearray, i: int) -> None:
    bf[i >> 3] |= 0x80 >> (i & 7)


def _concat(slices: Sequence[bytes], ranges: Sequence[tuple], n_pieces: int) -> bytearray:
    out = bytearray((n_pieces + 7) // 8)
    for (first, count), sl in zip(ranges, slices):
        if count:
            out[first // 8:first // 8 + len(sl)] = sl
    return out


_ctx_cache: dict = {}          # (device, slot) -> (Context, Lock)
_ctx_lock = threading.Lock()


@contextmanager
def _context(device: int, slot: int = 0):
    """The cached context of (device, shard slot), held exclusively for one whole job.  Device
    memory is reused across calls.  Concurrent shards of one call never share a context (a device
    may appear several times in `devices`).  Concurrent CALLS (threads, the async wrappers) take
    turns: a job's set_layout -> set_digests -> stage -> verify sequence is never interleaved with
    another job's."""
    with _ctx_lock:
        e = _ctx_cache.get((device, slot))
        if e is None:
            e = (_native.Context(device), threading.Lock())
            _ctx_cache[(device, slot)] = e
    ctx, lock = e
    with lock:
        yield ctx


def release_contexts() -> None:
    """Free every cached context (its HBM payload buffer and pinned staging ring).  The next call
    creates new ones.  Waits for jobs still running on them."""
    with _ctx_lock:
        entries = list(_ctx_cache.values())
        _ctx_cache.clear()
    for ctx, lock in entries:
        with lock:
            ctx.close()


def _devices(devices) -> List[int]:
    if devices is None:
        return [0]
    if isinstance(devices, int):
        return list(range(devices))
    return list(devices)


def _run_shards(devs: List[int], n_pieces: int, fn):
    """fn(ctx, first, count) for each shard, one thread per shard (ctypes releases the GIL)."""
    ranges = shard_ranges(n_pieces, len(devs))

    def run(slot: int, first: int, count: int):
        with _context(devs[slot], slot) as ctx:
            return fn(ctx, first, count)

    if len(devs) == 1:
        return ranges, [run(0, *ranges[0])]
    with ThreadPoolExecutor(len(devs)) as ex:
        futs = [ex.submit(run, s, f, n) for s, (f, n) in enumerate(ranges)]
        return ranges, [f.result() for f in futs]


def verify_pieces(info: InfoDict, storage, devices=None) -> bytearray:
    """verifyPieces(info, storage): have-bitfield of every piece read through `storage`
    (a torrent_amd.storage.Storage, i.e. the reference's Storage over any StorageMethod)."""
    P, L = info.n_pieces, info.piece_length

    def shard(ctx, first: int, count: int) -> bytes:
        ctx.set_layout(info.length, L, P, first, count)
        ctx.set_digests(info.pieces_raw)
        avail = bytearray((count + 7) // 8)
        per_batch = max(1, _STAGE_BATCH_BYTES // max(1, L))
        j = 0
        while j < count:
            k = min(per_batch, count - j)
            buf = bytearray(k * L)
            hi = 0
            for q in range(k):
                i = first + j + q
                n = piece_length(i, info)
                data = storage.get(i * L, n)  # storage.ts:50-65; None => unreadable => bit 0
                if data is None:
                    continue
                buf[q * L:q * L + n] = data
                hi = q * L + n
                _set_bit(avail, j + q)
            if hi:
                ctx.stage((first + j) * L, memoryview(buf)[:hi])
            j += k
        return ctx.verify(avail)

    if P == 0:
        return bytearray()
    ranges, slices = _run_shards(_devices(devices), P, shard)
    return _concat(slices, ranges, P)


def verify_payload(info: InfoDict, payload, devices=None, resident: bool = True,
                   avail: Optional[bytes] = None) -> bytearray:
    """Verify a linear payload already in host memory (the concatenation of info.files in
    order).  resident=True stages it into HBM and verifies there; resident=False streams it
    column by column over PCIe (tv_verify_host, the end-to-end resume-check path)."""
    P, L = info.n_pieces, info.piece_length
    mv = memoryview(payload).cast("B")

    def shard(ctx, first: int, count: int) -> bytes:
        ctx.set_layout(info.length, L, P, first, count)
        ctx.set_digests(info.pieces_raw)
        av = None
        if avail is not None:
            av = bytearray((count + 7) // 8)
            for j in range(count):
                i = first + j
                if (avail[i >> 3] >> (7 - (i & 7))) & 1:
                    _set_bit(av, j)
        lo = min(first * L, len(mv))
        hi = min((first + count) * L, len(mv))
        if resident:
            if hi > lo:
                ctx.stage(lo, mv[lo:hi])
            # pieces whose bytes are not all present are unreadable
            have = bytearray((count + 7) // 8)
            for j in range(count):
                i = first + j
                if i * L + piece_length(i, info) <= len(mv):
                    _set_bit(have, j)
            if av is not None:
                have = bytearray(a & b for a, b in zip(have, av))
            return ctx.verify(have)
        return ctx.verify_host(mv[lo:hi] if hi > lo else b"", av)

    if P == 0:
        return bytearray()
    ranges, slices = _run_shards(_devices(devices), P, shard)
    return _concat(slices, ranges, P)


def _files_shard(ctx, info: InfoDict, storage, first: int, count: int, threads: int,
                 batch_bytes: int, read_chunk: int = 8 << 20, direct_min: Optional[int] = None) -> bytearray:
    """Stage the shard's pieces from files into HBM and return the shard's readability bits.

    The shard's linear range is mapped to file segments exactly as Storage.get maps it
    (storage.ts:89-137).  Then:
      * a segment of >= direct_min bytes is staged by tv_stage_file: its page-cache pages are mapped,
        registered read-only and DMA'd straight to HBM (no host copy), on a thread of its own;
      * shorter segments that are adjacent in the linear space are grouped into runs of at most
        batch_bytes; a run is read by parallel preads (read_chunk pieces, so all threads copy even
        when one file covers the run) into one of two alternating page-locked buffers and DMA'd
        while the next run is read.
    A piece touching a missing or short file is unreadable (fsStorage.get -> null,
    storage.ts:150-172); zero-length segments succeed; missing files are never created."""
    import os
    L = info.piece_length
    if direct_min is None:
        direct_min = _DIRECT_MIN_BYTES
    avail = bytearray(b"\xff" * ((count + 7) // 8))
    if count % 8:
        avail[-1] = (0xFF00 >> (count % 8)) & 0xFF
    fds: dict = {}
    lock = threading.Lock()

    def fd_of(path):
        key = os.path.join(*path)
        with lock:
            if key not in fds:
                try:
                    fd = os.open(key, os.O_RDONLY)
                    fds[key] = (fd, os.fstat(fd).st_size)
                except OSError:
                    fds[key] = (None, -1)
            return fds[key]

    def clear(j_lo: int, j_hi: int) -> None:   # shard-relative pieces [j_lo, j_hi] unreadable
        with lock:
            for j in range(max(0, j_lo), min(count - 1, j_hi) + 1):
                avail[j >> 3] &= ~(0x80 >> (j & 7)) & 0xFF

    lo = first * L
    last = first + count - 1
    hi = last * L + piece_length(last, info)
    # pieces whose bytes extend past the last file (more digests than data) are unreadable
    j = count - 1
    while j >= 0 and (first + j) * L + piece_length(first + j, info) > info.length:
        clear(j, j)
        j -= 1
    span = max(0, min(hi, info.length) - lo)
    segs = storage.segments(lo, span) if span else []
    if segs is None:                  # unmappable (Storage.get -> null for every piece)
        clear(0, count - 1)
        segs = []

    direct: list = []                 # (path, file offset, shard-relative start, n)
    runs: list = []                   # [start, n, [(fd, file offset, run-relative start, n)]]
    run_cap = max(1, batch_bytes)
    for path, foff, n, start in segs:
        if n == 0:
            continue
        fd, size = fd_of(path)
        if fd is None or foff + n > size:
            clear(start // L, (start + n - 1) // L)
            continue
        if n >= direct_min:
            direct.append((os.path.join(*path), foff, start, n))
            continue
        while n:                      # a segment longer than a run is cut across runs
            cur = runs[-1] if runs else None
            if cur is not None and cur[0] + cur[1] == start and cur[1] < run_cap:
                k = min(n, run_cap - cur[1])
                cur[2].append((fd, foff, start - cur[0], k))
                cur[1] += k
            else:
                k = min(n, run_cap)
                runs.append([start, k, [(fd, foff, 0, k)]])
            foff, start, n = foff + k, start + k, n - k

    def stage_direct() -> None:
        for path, foff, start, n in direct:
            if not ctx.stage_file(path, foff, lo + start, n):
                clear(start // L, (start + n - 1) // L)

    def read_run(run, buf) -> None:
        start0, _, parts = run
        tasks = []
        for fd, foff, rel, n in parts:
            for s0 in range(0, n, read_chunk):
                tasks.append((fd, foff + s0, rel + s0, min(read_chunk, n - s0)))

        def one(t):
            fd, foff, rel, c = t
            try:
                got = os.preadv(fd, [buf.mv[rel:rel + c]], foff)
            except OSError:
                got = -1
            return None if got == c else (rel, c)

        for r in pool.map(one, tasks):
            if r is not None:
                rel, c = r
                clear((start0 + rel) // L, (start0 + rel + c - 1) // L)

    pool = ThreadPoolExecutor(max(1, threads))
    stager = ThreadPoolExecutor(2)    # one thread for direct segments, one for run DMAs
    bufs = []
    try:
        dfut = stager.submit(stage_direct) if direct else None
        if runs:
            size = max(r[1] for r in runs)
            bufs = [_native.PinnedBuffer(size)] + ([_native.PinnedBuffer(size)] if len(runs) > 1 else [])
        fut = None
        for b, run in enumerate(runs):
            buf = bufs[b & 1]
            read_run(run, buf)
            if fut is not None:
                fut.result()           # the other buffer's DMA is done before it is reused
            fut = stager.submit(ctx.stage, lo + run[0], buf.mv[:run[1]])
        if fut is not None:
            fut.result()
        if dfut is not None:
            dfut.result()
    finally:
        stager.shutdown()
        pool.shutdown()
        for fd, _ in fds.values():
            if fd is not None:
                os.close(fd)
        for bb in bufs:
            bb.close()
    return avail


def verify_files(info: InfoDict, dir_path: str, devices=None, threads: int = 16,
                 batch_bytes: int = 256 << 20, read_chunk: int = 8 << 20,
                 direct_min: Optional[int] = None) -> bytearray:
    """Resume check from disk: the have-bitfield of the files under dir_path,
    laid out as Storage(fs_storage, info, dir_path) maps them (storage.ts:89-137; single-file
    torrents are [dir, name], multi-file [dir, *path] without info.name).

    Same bits as verify_pieces(info, Storage(fs_storage, info, dir_path)), without fsStorage.get's
    side effect of creating missing files.  Long file segments (>= direct_min bytes, default 32 MiB)
    are DMA'd to HBM straight from the page cache; shorter ones are read by parallel preads into
    page-locked buffers (see _files_shard) instead of one open/seek/read per piece."""
    from .storage import Storage, fs_storage

    P, L = info.n_pieces, info.piece_length
    storage = Storage(fs_storage, info, dir_path)

    def shard(ctx, first: int, count: int) -> bytes:
        ctx.set_layout(info.length, L, P, first, count)
        ctx.set_digests(info.pieces_raw)
        if count == 0:
            return b""
        return ctx.verify(_files_shard(ctx, info, storage, first, count, threads, batch_bytes, read_chunk,
                                       direct_min))

    if P == 0:
        return bytearray()
    ranges, slices = _run_shards(_devices(devices), P, shard)
    return _concat(slices, ranges, P)


def hash_files(info: InfoDict, dir_path: str, devices=None, threads: int = 16,
               batch_bytes: int = 256 << 20, read_chunk: int = 8 << 20,
               direct_min: Optional[int] = None) -> bytes:
    """Creation mode from disk: the `pieces` string of the files info describes under dir_path
    (info.pieces is ignored; only the geometry is used).  Raises if a file is missing or short."""
    from .storage import Storage, fs_storage

    L = info.piece_length
    P = -(-info.length // L) if info.length else 0
    storage = Storage(fs_storage, info, dir_path)

    def shard(ctx, first: int, count: int) -> bytes:
        ctx.set_layout(info.length, L, P, first, count)
        if count == 0:
            return b""
        avail = _files_shard(ctx, info, storage, first, count, threads, batch_bytes, read_chunk,
                             direct_min)
        full = bytearray(b"\xff" * ((count + 7) // 8))
        if count % 8:
            full[-1] = (0xFF00 >> (count % 8)) & 0xFF
        if avail != full:
            raise FileNotFoundError("hash_files: a file is missing or shorter than its declared length")
        return ctx.hash()

    if P == 0:
        return b""
    _, slices = _run_shards(_devices(devices), P, shard)
    return b"".join(slices)


def verify_piece(info: InfoDict, index: int, data) -> bool:
    """verifyPiece(info, index, bytes): SHA-1(bytes) == info.pieces[index] for a piece of the
    right length (piece.ts:16-19).  Raises ValueError for an index out of range (piece.ts:22)."""
    if index < 0 or index >= info.n_pieces:
        raise ValueError(f"verify_piece: invalid piece index {index}")
    n = memoryview(data).nbytes
    if n != piece_length(index, info) or len(info.pieces[index]) != 20 or n == 0:
        return False
    with _context(0) as ctx:
        ctx.set_layout(n, n, 1, 0, 1)
        ctx.set_digests(bytes(info.pieces[index]))
        ctx.stage(0, data)
        return bool(ctx.verify()[0] & 0x80)


def hash_pieces(payload, piece_length_: int, devices=None) -> bytes:
    """Creation mode: the `pieces` byte string for a linear payload (make_torrent.ts:147-173;
    multi-file payloads are the files concatenated in order, make_torrent.ts:62-113)."""
    mv = memoryview(payload).cast("B")
    total = len(mv)
    P = -(-total // piece_length_) if total else 0

    def shard(ctx, first: int, count: int) -> bytes:
        ctx.set_layout(total, piece_length_, P, first, count)
        lo, hi = first * piece_length_, min(total, (first + count) * piece_length_)
        if hi > lo:
            ctx.stage(lo, mv[lo:hi])
        return ctx.hash()

    if P == 0:
        return b""
    _, slices = _run_shards(_devices(devices), P, shard)
    return b"".join(slices)


async def verify_pieces_async(info: InfoDict, storage, devices=None) -> bytearray:
    return await asyncio.to_thread(verify_pieces, info, storage, devices)


async def verify_piece_async(info: InfoDict, index: int, data) -> bool:
    return await asyncio.to_thread(verify_piece, info, index, data)
