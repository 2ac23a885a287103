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

Device memory.  The bulk calls take `budget` (bytes of HBM the payload may use per device; None = the
GPU's free memory less a margin).  A shard larger than it is verified in windows of pieces that fit, each
hashed while the next one stages (tv_set_layout's windowed layout): no torrent is too large for a GPU.  Where such
windows would lose (a window pays one piece's serial SHA-1), verify_files (_stream_wins) and verify_payload stream
the shard instead, windows x columns within the budget through the bounded ring.

Public API (names follow the reference's camelCase surface, snake_cased):
    verify_pieces(info, storage, devices=None) -> bytearray         (verifyPieces)
    verify_piece(info, index, data) -> bool                         (verifyPiece)
    verify_payload(info, payload, devices=None, resident=None) -> bytearray
    verify_stream(info, read, devices=None) -> bytearray             (bounded-ring resume check)
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
from ._cpu import shard_threads
from .piece import piece_length
from .storage import copy_bytes

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
# verify_piece's context slot: a one-piece layout on a bulk call's context (slot 0) would free its payload
# (tv_set_layout keeps an allocation only while the new geometry is at least half of it) and the next bulk
# call would allocate it again
_PIECE_SLOT = -1
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


def context_counters() -> dict:
    """{(device, slot): {payload_allocs, device_allocs, payload_bytes, device_bytes}} of the cached contexts
    (tv_get_counter): how often each had to allocate device memory, and what it holds now."""
    with _ctx_lock:
        entries = list(_ctx_cache.items())
    out = {}
    for key, (ctx, lock) in entries:
        with lock:
            out[key] = {name: ctx.counter(k) for name, k in (
                ("payload_allocs", _native.TV_COUNTER_PAYLOAD_ALLOCS), ("device_allocs", _native.TV_COUNTER_DEVICE_ALLOCS),
                ("payload_bytes", _native.TV_COUNTER_PAYLOAD_BYTES), ("device_bytes", _native.TV_COUNTER_DEVICE_BYTES),
                ("window_pieces", _native.TV_COUNTER_WINDOW_PIECES), ("windows", _native.TV_COUNTER_WINDOWS),
                ("budget", _native.TV_COUNTER_BUDGET))}
    return out


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


def _layout(ctx, info_or_len, L: int, P: int, first: int, count: int, budget: Optional[int]) -> None:
    """set_layout with this call's device budget (the contexts are cached: every call sets its own)."""
    ctx.set_option(_native.TV_OPT_RESIDENT_BUDGET, int(budget or 0))
    total = info_or_len if isinstance(info_or_len, int) else info_or_len.length
    ctx.set_layout(total, L, P, first, count)


def _batch_buffers(ctx, nbytes: int) -> list:
    """Two page-locked batch buffers of `ctx` holding >= nbytes each (kept on the cached context and reused):
    reads land in them and tv_stage DMAs them straight to HBM, with no copy through the staging ring."""
    bufs = getattr(ctx, "_batch_bufs", None)
    if bufs is None or bufs[0].nbytes < nbytes:
        for b in bufs or ():
            b.close()
        ctx._batch_bufs = None
        bufs = ctx._batch_bufs = [_native.PinnedBuffer(nbytes) for _ in range(2)]
    return bufs


def _chunked_map(pool, fn, n: int, parts: int) -> list:
    """[fn(0), .., fn(n - 1)] with the indices split into `parts` contiguous runs, one pool task per run (pool None:
    in this thread).  One task per index costs a Future, a queue hand-off and a thread wake-up each, which on
    10,000 small files cost more than the reads (tools/threads_sweep.py)."""
    if pool is None or parts <= 1 or n <= 1:
        return [fn(q) for q in range(n)]
    parts = min(parts, n)
    bounds = [n * r // parts for r in range(parts + 1)]
    out = []
    for run in pool.map(lambda r: [fn(q) for q in range(bounds[r], bounds[r + 1])], range(parts)):
        out.extend(run)
    return out


_node_of: dict = {}            # device -> NUMA node of its GPU (None: unknown), from the library (TV_COUNTER_NUMA_NODE)


def _device_node(device: int, slot: int) -> Optional[int]:
    if device not in _node_of:
        with _context(device, slot) as ctx:
            v = ctx.counter(_native.TV_COUNTER_NUMA_NODE)
        _node_of[device] = None if v >= (1 << 63) else int(v)
    return _node_of[device]


def _run_shards(devs: List[int], n_pieces: int, fn):
    """fn(ctx, first, count) for each shard, one thread per shard (ctypes releases the GIL).  The shards share
    the process's CPUs: each context gets its part (ctx.thread_budget, also set as TV_OPT_FILE_THREADS), so
    devices=[0..7] does not start 8 x 16 reader threads on a 16-CPU share (_cpu.shard_threads)."""
    ranges = shard_ranges(n_pieces, len(devs))
    active = [s for s, (_, count) in enumerate(ranges) if count]
    budget = dict(zip(active, shard_threads([_device_node(devs[s], s) for s in active])))

    def run(slot: int, first: int, count: int):
        if count == 0:       # a trailing empty shard (P < 8 x devices): no context, no bits
            return b""
        with _context(devs[slot], slot) as ctx:
            ctx.thread_budget = budget[slot]
            ctx.set_option(_native.TV_OPT_FILE_THREADS, budget[slot])
            return fn(ctx, first, count)

    if len(devs) == 1:
        return ranges, [run(0, *ranges[0])]
    with ThreadPoolExecutor(len(devs)) as ex:
        futs = [ex.submit(run, s, f, n) for s, (f, n) in enumerate(ranges)]
        return ranges, [f.result() for f in futs]


# Python reader threads of the Storage paths (verify_pieces, verify_stream): each Storage.get is Python work under
# the GIL around its open / pread / copy, so past a few threads they contend more than they overlap -- 4 was the
# fastest or within noise of it on cfg3's 10,000 files and on 16 GiB in one and in 64 files, warm, for both paths
# (tools/threads_sweep.py, profiles/r04/threads_sweep.jsonl).  (verify_files reads in the library's own threads.)
_STORAGE_THREADS = 4


def _storage_threads(ctx, threads: Optional[int]) -> int:
    """Reader threads of a Storage path: the caller's count as given, or by default _STORAGE_THREADS capped at the
    shard's part of the process's CPUs (ctx.thread_budget; ADVICE r05: an explicit count is never cut silently)."""
    if threads is None:
        return max(1, min(_STORAGE_THREADS, ctx.thread_budget))
    return max(1, int(threads))


def verify_pieces(info: InfoDict, storage, devices=None, threads: Optional[int] = None,
                  budget: Optional[int] = None) -> bytearray:
    """verifyPieces(info, storage): have-bitfield of every piece read through `storage`
    (a torrent_amd.storage.Storage, i.e. the reference's Storage over any StorageMethod).  The gets
    of a batch are in flight together on `threads` threads, as ts/verify.ts keeps them outstanding
    with Promise.all (make_torrent.ts:96,111 does the same); threads=1 reads them one by one.  threads=None (the
    default): _STORAGE_THREADS, capped at the shard's part of the process's CPUs (ctx.thread_budget); an explicit
    count is used as given (e.g. more threads for a Storage whose gets mostly wait).
    Reads and staging overlap: batch k + 1 is read (into the other of two page-locked buffers) while batch
    k is DMA'd to HBM (and, on a windowed layout, while the windows before it hash); each reader thread
    copies its piece into the batch buffer itself, without the GIL."""
    P, L = info.n_pieces, info.piece_length

    def shard(ctx, first: int, count: int) -> bytes:
        _layout(ctx, info, L, P, first, count, budget)
        ctx.set_digests(info.pieces_raw)
        avail = bytearray((count + 7) // 8)
        per_batch = max(1, min(count, _STAGE_BATCH_BYTES // max(1, L)))

        def get(i: int, base: int) -> int:
            """Piece i into the batch buffer at `base` (+ its slot); its length, or 0 when unreadable."""
            n = piece_length(i, info)
            data = storage.get(i * L, n)         # storage.ts:50-65; None => bit 0
            # (Storage.get returns exactly the length asked or null; any other length is unreadable too,
            # as in verify_stream -- it must not shift the batch buffer's later pieces)
            if data is None or len(data) != n:
                return 0
            copy_bytes(base, data, n)
            return n

        bufs = _batch_buffers(ctx, per_batch * L)
        nthr = _storage_threads(ctx, threads)
        with ThreadPoolExecutor(nthr) as pool, ThreadPoolExecutor(1) as stager:
            staging = None              # the previous batch's stage (it reads the other buffer)
            j, b = 0, 0
            try:
                while j < count:
                    k = min(per_batch, count - j)
                    buf = bufs[b]       # its last stage (two batches ago) finished before `staging` began
                    hi = 0
                    got = _chunked_map(pool, lambda q: get(first + j + q, buf.ptr + q * L), k, nthr)
                    for q, n in enumerate(got):
                        if n:           # (an unreadable piece's slot keeps stale bytes: never a readable piece)
                            hi = q * L + n
                            _set_bit(avail, j + q)
                    if staging is not None:
                        staging.result()
                        staging = None
                    if hi:
                        staging = stager.submit(ctx.stage, (first + j) * L, buf.mv[:hi])
                    j += k
                    b ^= 1
            finally:
                if staging is not None:
                    staging.result()
        return ctx.verify(avail)

    if P == 0:
        return bytearray()
    ranges, slices = _run_shards(_devices(devices), P, shard)
    return _concat(slices, ranges, P)


def verify_payload(info: InfoDict, payload, devices=None, resident: Optional[bool] = None,
                   avail: Optional[bytes] = None, budget: Optional[int] = None) -> bytearray:
    """Verify a linear payload already in host memory (the concatenation of info.files in
    order).  resident=True stages it into HBM and verifies there (in windows of whole pieces when the shard exceeds
    `budget`); resident=False streams it column by column over PCIe (tv_verify_host, the end-to-end
    resume-check path; under a `budget`, windows x columns within it).  None (default): resident when the shard fits
    the budget, else streamed -- from host memory the stream beats windows of whole pieces at every budget (54.9-55.5
    GB/s at 0.25-2 GiB against 14.4 / 28.3 / 51.6 / 53.8, profiles/r06/window_bench_payload_cols3.jsonl)."""
    P, L = info.n_pieces, info.piece_length
    mv = memoryview(payload).cast("B")

    def shard(ctx, first: int, count: int) -> bytes:
        streamed = resident is False or (resident is None and _exceeds(L, count, budget))
        if streamed:            # the streamed path needs no resident payload (tv_verify_host)
            ctx.set_option(_native.TV_OPT_RESIDENT, 0)
        try:
            _layout(ctx, info, L, P, first, count, budget)
        finally:
            ctx.set_option(_native.TV_OPT_RESIDENT, 1)
        ctx.set_digests(info.pieces_raw)
        av = _shard_avail(avail, first, count)
        lo = min(first * L, len(mv))
        hi = min((first + count) * L, len(mv))
        if not streamed:
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


def _shard_avail(avail: Optional[bytes], first: int, count: int) -> Optional[bytearray]:
    """Shard-relative slice of a torrent-wide MSB-first availability bitfield (None = all readable)."""
    if avail is None:
        return None
    av = bytearray((count + 7) // 8)
    for j in range(count):
        i = first + j
        if (avail[i >> 3] >> (7 - (i & 7))) & 1:
            _set_bit(av, j)
    return av


def verify_stream(info: InfoDict, read, devices=None, avail: Optional[bytes] = None, chunk: int = 0,
                  threads: Optional[int] = None) -> bytearray:
    """End-to-end resume check through the library's BOUNDED pinned ring (tv_stream_*; SURVEY 8d config 5:
    the resume flow Client.add -> verify -> Torrent.bitfield -> sendBitfield, client.ts:53-67,
    torrent.ts:56-60,101).  No resident payload and no whole-shard host buffer.  By default (chunk=0) each
    request row is a WHOLE piece (TV_OPT_STREAM_ROWS; pieces of up to 64 MiB), so a piece costs one
    read(linear_offset, length) -> bytes | None -- Storage.get's shape (storage.ts:50-65), so a Storage's
    bound .get can be passed, and fsStorage.get opens each file once per piece; the library hashes windows of
    up to 4 GiB of pieces as they arrive.  chunk=C > 0 asks for the shard column by column instead (bytes
    [c*C, c*C + C) of every piece; all of the shard's pieces in each launch).  None makes that piece
    unreadable (bit 0); a piece is readable iff every slice of it reads.  Host memory in flight: 3 x 64 MiB
    per device, whatever the size.  The reads of a request are in flight together on `threads` threads (as
    verify_pieces; threads=1 reads them one by one; None: the default and CPU cap of verify_pieces), each writing its
    own row of the slot."""
    P, L = info.n_pieces, info.piece_length

    def shard(ctx, first: int, count: int) -> bytes:
        ctx.set_option(_native.TV_OPT_RESIDENT, 0)       # no resident payload for a streamed check
        try:
            # (a budget an earlier call left on the cached context would cap the row windows: ADVICE r04)
            ctx.set_option(_native.TV_OPT_RESIDENT_BUDGET, 0)
            ctx.set_option(_native.TV_OPT_STREAM_CHUNK, chunk)
            ctx.set_option(_native.TV_OPT_STREAM_ROWS, 0 if chunk else 1)
            ctx.set_layout(info.length, L, P, first, count)
            ctx.set_digests(info.pieces_raw)
        finally:
            ctx.set_option(_native.TV_OPT_RESIDENT, 1)
        ctx.stream_begin(_shard_avail(avail, first, count))
        nthr = _storage_threads(ctx, threads)
        pool = ThreadPoolExecutor(nthr) if nthr > 1 else None
        try:
            while True:
                req = ctx.stream_next()
                if not req.rows:
                    break

                def fill(q: int, req=req):
                    """Row q into the slot (copied by this reader thread, without the GIL); returns the piece
                    index when it is unreadable."""
                    n = ctx.row_bytes(req, q)
                    if n == 0:
                        return None
                    i = req.piece + q
                    data = read(i * L + req.offset, n)
                    if data is None or len(data) != n:
                        return i
                    copy_bytes(req.slot + q * req.width, data, n)
                    return None

                for i in _chunked_map(pool, fill, req.rows, nthr):
                    if i is not None:
                        ctx.stream_unreadable(i)
                ctx.stream_commit(req)
            return ctx.stream_end()
        except BaseException:
            ctx.stream_abort()
            raise
        finally:
            if pool is not None:
                pool.shutdown()
            ctx.set_option(_native.TV_OPT_STREAM_CHUNK, 0)
            ctx.set_option(_native.TV_OPT_STREAM_ROWS, 0)

    if P == 0:
        return bytearray()
    ranges, slices = _run_shards(_devices(devices), P, shard)
    return _concat(slices, ranges, P)


def _files_shard(ctx, info: InfoDict, storage, first: int, count: int, threads: int = 16,
                 direct_min: Optional[int] = None, status_out: Optional[list] = None,
                 open_rw: bool = True) -> bytearray:
    """Stage the shard's pieces from files into HBM and return the shard's readability bits.

    The shard's linear range is mapped to file segments exactly as Storage.get maps it
    (storage.ts:89-137), and ALL segments go to the library in one tv_stage_files call: segments of
    >= direct_min bytes (default 32 MiB) are DMA'd from the page cache (tv_stage_file's path), shorter
    ones are read by `threads` library threads into pinned slots, one DMA per run of adjacent bytes.
    The library marks the unreadable pieces itself, exactly as Storage.get(i * L, len_i) would return null
    (storage.ts:50-65,150-172): a piece with a byte in a missing, unopenable or too-short part of a file,
    and a piece whose zero-length segment (storage.ts:109-110) names a path fsStorage.get could not open;
    a short file's pieces before its end stay readable.  Missing files are never created.  `status_out`, if
    given, receives the per-segment statuses (hash_files raises on any failure).  open_rw: files are opened
    read + write as fsStorage.get opens them (storage.ts:28-32,158); False opens them read-only, as
    make_torrent.ts:78 opens its sources (hash_files)."""
    L = info.piece_length
    avail = bytearray(b"\xff" * ((count + 7) // 8))
    if count % 8:
        avail[-1] = (0xFF00 >> (count % 8)) & 0xFF

    def clear(j_lo: int, j_hi: int) -> None:   # shard-relative pieces [j_lo, j_hi] unreadable
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
    # the n_bytes > 0 segments of Storage.segments(lo, span), as arrays (same walk, vectorised)
    segs = storage.segment_arrays(lo, span) if span else None
    if span and segs is None:         # unmappable (Storage.get -> null for every piece)
        clear(0, count - 1)
    if segs is None:
        return avail
    import numpy as np

    k, foff, nbytes, start = segs
    lin = start + lo
    # the walk's zero-length segments too: the library checks their open as fsStorage.get would make it
    zk, zfoff, zlin = storage.zero_length_segments(lo, span, L)
    if len(zk):
        k, foff, lin = np.concatenate([k, zk]), np.concatenate([foff, zfoff]), np.concatenate([lin, zlin])
        nbytes = np.concatenate([nbytes, np.zeros(len(zk), np.int64)])
    if len(k) == 0:
        return avail
    # a path holding a NUL cannot be opened (Deno.open throws, so fsStorage.get's piece is null, storage.ts:157-170):
    # it goes as "", which the library cannot open either (ts/verify.ts does the same)
    paths = [p if "\0" not in p else "" for p in storage.file_paths()]
    ctx.set_option(_native.TV_OPT_FILE_THREADS, max(1, threads))
    ctx.set_option(_native.TV_OPT_OPEN_RW, 1 if open_rw else 0)
    ctx.set_option(_native.TV_OPT_FILE_DIRECT_MIN, _DIRECT_MIN_BYTES if direct_min is None else direct_min)
    # a failed segment's pieces are marked inside the library (tv_verify reports them 0): from the piece
    # holding its first unreadable byte on, as Storage.get reads piece by piece; the statuses are informational
    status = ctx.stage_files([paths[i] for i in k.tolist()], foff, lin, nbytes)
    if status_out is not None:
        status_out.extend(status)
    return avail


def _exceeds(L: int, count: int, budget: Optional[int]) -> bool:
    """Whether a shard's padded payload (tv_set_layout: count x (L rounded up to 64 + 256) + 256 bytes) exceeds a
    device budget (None: the library's automatic one, never exceeded here)."""
    return bool(budget) and count * (-(-L // 64) * 64 + 256) + 256 > budget


def _stream_wins(L: int, count: int, budget: Optional[int]) -> bool:
    """Whether a file-backed shard verifies faster in streamed columns than in windows of whole pieces under this
    device budget: only when the shard does not fit it, and each window (two of three buffers hashing at once) would
    cost more than staging -- a window pays one piece's serial SHA-1 (~11.8 ms per MiB of piece), so windows keep up
    with ~50 GB/s of staging only from ~0.9 GB of budget per MiB of piece length (profiles/r06/window_bench_stream.jsonl:
    0.5 GiB, 1 MiB pieces: columns 47.5 GB/s against windows 28.3; 1 GiB 50.6 / 50.4; 2 GiB 48.9 / 51.7)."""
    return _exceeds(L, count, budget) and budget < 0.9e9 * L / (1 << 20)


def _stream_files_shard(ctx, info: InfoDict, storage, first: int, count: int, threads: int,
                        budget: Optional[int]) -> bytes:
    """A shard's resume check from its files through the bounded ring (tv_stream_file_table): no resident payload,
    two device chunk buffers within the budget (columns of windows of >= 2,048 pieces), the library's readers filling
    each column from the file table."""
    L, P = info.piece_length, info.n_pieces
    ctx.set_option(_native.TV_OPT_RESIDENT, 0)
    try:
        # the library sizes windows x columns to the budget (tv_stream_file_table)
        ctx.set_option(_native.TV_OPT_RESIDENT_BUDGET, int(budget or 0))
        ctx.set_option(_native.TV_OPT_STREAM_CHUNK, 0)
        ctx.set_option(_native.TV_OPT_STREAM_ROWS, 0)
        ctx.set_layout(info.length, L, P, first, count)
        ctx.set_digests(info.pieces_raw)
    finally:
        ctx.set_option(_native.TV_OPT_RESIDENT, 1)
    if count == 0:
        return b""
    ctx.set_option(_native.TV_OPT_FILE_THREADS, max(1, threads))
    ctx.set_option(_native.TV_OPT_OPEN_RW, 1)
    lengths = [info.length] if info.files is None else [f.length for f in info.files]
    paths = [p if "\0" not in p else "" for p in storage.file_paths()]
    bits, _ = ctx.stream_file_table(lengths, paths)
    return bits


def verify_files(info: InfoDict, dir_path: str, devices=None, threads: Optional[int] = None,
                 direct_min: Optional[int] = None, budget: Optional[int] = None,
                 stream: Optional[bool] = None) -> bytearray:
    """Resume check from disk: the have-bitfield of the files under dir_path,
    laid out as Storage(fs_storage, info, dir_path) maps them (storage.ts:89-137; single-file
    torrents are [dir, name], multi-file [dir, *path] without info.name).

    Same bits as verify_pieces(info, Storage(fs_storage, info, dir_path)), without fsStorage.get's
    side effect of creating missing files, and with every file segment of a shard staged by ONE
    tv_stage_files call (see _files_shard) instead of one open/seek/read per piece.  threads: the library's
    reader threads per shard (default: the shard's part of the process's CPUs, _cpu.shard_threads).  budget: device
    bytes the shard's payload may take (default: the GPU's free memory less a margin); a shard above it is held in
    windows of whole pieces, or -- stream=True, or by default where windows would cost more than staging
    (_stream_wins) -- read through the bounded ring in columns sized to the budget (tv_stream_file_table)."""
    from .storage import Storage, fs_storage

    P, L = info.n_pieces, info.piece_length
    storage = Storage(fs_storage, info, dir_path)

    def shard(ctx, first: int, count: int) -> bytes:
        if stream or (stream is None and _stream_wins(L, count, budget)):
            return _stream_files_shard(ctx, info, storage, first, count, threads or ctx.thread_budget, budget)
        _layout(ctx, info, L, P, first, count, budget)
        ctx.set_digests(info.pieces_raw)
        if count == 0:
            return b""
        return ctx.verify(_files_shard(ctx, info, storage, first, count, threads or ctx.thread_budget, direct_min))

    if P == 0:
        return bytearray()
    ranges, slices = _run_shards(_devices(devices), P, shard)
    return _concat(slices, ranges, P)


def hash_files(info: InfoDict, dir_path: str, devices=None, threads: Optional[int] = None,
               direct_min: Optional[int] = None, budget: Optional[int] = None) -> bytes:
    """Creation mode from disk: the `pieces` string of the files info describes under dir_path
    (info.pieces is ignored; only the geometry is used).  Raises if a file is missing or short.  Files are
    opened read-only, as make_torrent.ts:78 opens its sources: the process need not be able to write them."""
    from .storage import Storage, fs_storage

    L = info.piece_length
    P = -(-info.length // L) if info.length else 0
    storage = Storage(fs_storage, info, dir_path)

    def shard(ctx, first: int, count: int) -> bytes:
        _layout(ctx, info, L, P, first, count, budget)
        if count == 0:
            return b""
        status: list = []
        avail = _files_shard(ctx, info, storage, first, count, threads or ctx.thread_budget, direct_min, status,
                             open_rw=False)
        full = bytearray(b"\xff" * ((count + 7) // 8))
        if count % 8:
            full[-1] = (0xFF00 >> (count % 8)) & 0xFF
        if avail != full or any(st != _native.TV_OK for st in status):
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
    with _context(0, _PIECE_SLOT) as ctx:      # its own context: never evicts a bulk call's payload
        _layout(ctx, n, n, 1, 0, 1, None)
        ctx.set_digests(bytes(info.pieces[index]))
        ctx.stage(0, data)
        return bool(ctx.verify()[0] & 0x80)


def hash_pieces(payload, piece_length_: int, devices=None, budget: Optional[int] = None) -> bytes:
    """Creation mode: the `pieces` byte string for a linear payload (make_torrent.ts:147-173;
    multi-file payloads are the files concatenated in order, make_torrent.ts:62-113)."""
    mv = memoryview(payload).cast("B")
    total = len(mv)
    P = -(-total // piece_length_) if total else 0

    def shard(ctx, first: int, count: int) -> bytes:
        _layout(ctx, total, piece_length_, P, first, count, budget)
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
