"""ctypes binding of libtorrent_verify.so (include/torrent_verify.h).

This is the Python analogue of the Deno `Deno.dlopen` binding in ts/verify.ts: the same
symbols, the same argument meaning, negative status -> exception.  There is no CPU fallback:
if the library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import sys
from typing import Optional

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TORRENT_VERIFY_LIB", os.path.join(_PKG, "libtorrent_verify.so"))

TV_OK = 0
TV_ERR_ARG = -1
TV_ERR_HIP = -2
TV_ERR_STATE = -3
TV_ERR_NOMEM = -4
TV_ERR_IO = -5

# public options (include/torrent_verify.h)
TV_OPT_STREAM_CHUNK = 3
TV_OPT_FILE_DIRECT_MIN = 7
TV_OPT_FILE_THREADS = 8
TV_OPT_RESIDENT = 10
TV_OPT_TWIN_FILL = 13
TV_OPT_RESIDENT_BUDGET = 16
TV_OPT_LIST_SLOTS = 17
TV_OPT_OPEN_RW = 18
TV_OPT_STREAM_ROWS = 19
TV_OPT_CLOCK_PROBE = 20

# measurement / test knobs (torrent_amd/csrc/tv_options_internal.h; tests and tools only)
TV_OPT_KERNEL = 1
TV_OPT_STRIDE_PAD = 2
TV_OPT_SPLIT_PAIRS = 4
TV_OPT_FILE_DIRECT = 5
TV_OPT_FILE_CHUNK = 6
TV_OPT_FILE_CONCURRENT = 9
TV_OPT_DEBUG_REBOUNCE = 11
TV_OPT_TWIN_PACK = 12
TV_OPT_TWIN_FILL_READS = 14
TV_OPT_NUMA_BIND = 15
TV_OPT_LANE_PAIRS = 21
TV_OPT_FILE_ODIRECT = 22
TV_OPT_FILE_CLOCK_RESET = 100
TV_COUNTER_FILE_CLOCK = 100
TV_COUNTER_COTENANT_VRAM = 120
TV_OPT_WIN_BUFS = 23
TV_OPT_FILE_BOUNCE = 25
TV_OPT_WIN_STREAMS = 24
TV_OPT_STREAM_COLD_WINDOW = 26
TV_OPT_STREAM_COLD_READERS = 27
TV_OPT_STREAM_COLD_REQ = 28
TV_COUNTER_WINDOW_BUFS = 122
TV_COUNTER_WINDOW_STREAMS = 123
WIN_BUFS_DEFAULT = 3    # tv_plan.h kWinBufsDefault: window buffers of a windowed layout
FILE_BOUNCE_DEFAULT = 2  # tv_ctx.h file_bounce: cold-read bounce readers per staging lane
TV_COUNTER_KFD_GPU_ID = 121
TV_FILE_PHASES = ("open", "map", "populate", "register", "read", "wait", "queue", "release", "drain", "small", "call",
                  "bytes_direct", "bytes_read", "bytes_odirect", "odirect_fallbacks", "odirect_errno")   # TV_FILE_PHASE_* / TV_FILE_BYTES_* in order

TV_COUNTER_PAYLOAD_ALLOCS = 1
TV_COUNTER_DEVICE_ALLOCS = 2
TV_COUNTER_PAYLOAD_BYTES = 3
TV_COUNTER_DEVICE_BYTES = 4
TV_COUNTER_LAST_WORKGROUPS = 5
TV_COUNTER_NUMA_NODE = 6
TV_COUNTER_RING_NODE = 7
TV_COUNTER_WINDOW_PIECES = 8
TV_COUNTER_WINDOWS = 9
TV_COUNTER_BUDGET = 10
TV_COUNTER_SLOTS_USED = 11
TV_COUNTER_LAST_CLOCK_KHZ = 12

TV_STREAM_RING_SLOTS = 3
TV_STREAM_SLOT_BYTES = 64 << 20

KERNEL_AUTO, KERNEL_LANE, KERNEL_SPLIT, KERNEL_TWIN = 0, 1, 2, 4   # (3 was MIX, removed)

_u64, _i64, _int, _p = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p


def build_id(path: Optional[str] = None) -> Optional[str]:
    """The source id compiled into the library file (torrent_amd/_build.py source_id; the TV_BUILD_ID= marker), or
    None for a library built without one."""
    import re
    try:
        with open(path or LIB_PATH, "rb") as f:
            m = re.search(rb"TV_BUILD_ID=([0-9a-f]{16})", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


class StreamReq(ctypes.Structure):
    """tv_stream_req (include/torrent_verify.h): rows [piece, piece+rows) x bytes [offset, offset+width)."""
    _fields_ = [("piece", _u64), ("rows", _u64), ("offset", _u64), ("width", _u64), ("slot", _p), ("seq", _u64)]


_REQ = ctypes.POINTER(StreamReq)

# every symbol include/torrent_verify.h declares: (name, restype, argtypes)
SYMBOLS = [
    ("tv_abi_version", _int, []),
    ("tv_device_count", _int, [ctypes.POINTER(_int)]),
    ("tv_cpu_share", _int, [ctypes.POINTER(ctypes.c_uint32)]),
    ("tv_create", _int, [ctypes.POINTER(_p), _int]),
    ("tv_destroy", None, [_p]),
    ("tv_last_error", _int, [_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("tv_set_layout", _int, [_p, _u64, _u64, _u64, _u64, _u64]),
    ("tv_set_digests", _int, [_p, _p, _u64]),
    ("tv_stage", _int, [_p, _u64, _p, _u64]),
    ("tv_stage_many", _int, [_p, _u64, _p, _p, _p]),
    ("tv_stage_file", _int, [_p, ctypes.c_char_p, _u64, _u64, _u64]),
    ("tv_stage_files", _int, [_p, _u64, _p, _p, _p, _p, _p]),
    ("tv_stage_file_table", _int, [_p, _u64, _p, _p, _u64, _p]),
    ("tv_stream_file_table", _int, [_p, _u64, _p, _p, _u64, _p, _p, _p]),
    ("tv_read", _int, [_p, _u64, _p, _u64]),
    ("tv_fill_synthetic", _int, [_p, _u64]),
    ("tv_verify", _int, [_p, _p, _p]),
    ("tv_verify_host", _int, [_p, _p, _u64, _p, _p]),
    ("tv_verify_list", _int, [_p, _p, _u64, _p]),
    ("tv_hash", _int, [_p, _p]),
    ("tv_stream_begin", _int, [_p, _p]),
    ("tv_stream_next", _int, [_p, _REQ]),
    ("tv_stream_commit", _int, [_p, _REQ]),
    ("tv_stream_commit_from", _int, [_p, _REQ, _p, _u64]),
    ("tv_stream_unreadable", _int, [_p, _u64]),
    ("tv_stream_end", _int, [_p, _p]),
    ("tv_stream_abort", _int, [_p]),
    ("tv_stream_fill_synthetic", _int, [_p, _REQ, _u64]),
    ("tv_set_option", _int, [_p, _int, _i64]),
    ("tv_get_option", _int, [_p, _int, ctypes.POINTER(_i64)]),
    ("tv_last_timing", _int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    ("tv_last_kernel", _int, [_p, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    ("tv_get_counter", _int, [_p, _int, ctypes.POINTER(_u64)]),
    ("tv_synchronize", _int, [_p]),
    ("tv_host_alloc", _int, [_u64, ctypes.POINTER(_p)]),
    ("tv_host_free", _int, [_p]),
    ("tv_host_register", _int, [_p, _u64]),
    ("tv_host_unregister", _int, [_p]),
]

_lib = None


class NativeError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"torrent_verify error {code}: {message}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load the HIP library.  Raises (never falls back) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -m torrent_amd._build` "
                              "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.tv_abi_version() != 1:
            raise ImportError("libtorrent_verify ABI version mismatch")
        _lib = L
    return _lib


def _addr(buf, writable: bool = False) -> tuple:
    """(void* address, keepalive) of a bytes-like object or None, never a copy: the library reads sources
    in place (a read-only buffer such as a slice of a 16 GiB `bytes` payload is not duplicated), and writes
    outputs in place, so a read-only buffer given as an output (`writable`) is a TypeError rather than a
    silent write into a temporary."""
    if buf is None:
        return None, None
    if isinstance(buf, bytes) and not writable:
        return ctypes.cast(ctypes.c_char_p(buf), _p).value, buf
    mv = memoryview(buf).cast("B")
    if mv.nbytes == 0:
        return None, None
    if mv.readonly:
        if writable:
            raise TypeError("the output buffer is read-only")
        import numpy as np
        a = np.frombuffer(mv, dtype=np.uint8)   # a view: the exporter's own bytes
        return a.ctypes.data, a
    c = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return ctypes.addressof(c), c


def device_count() -> int:
    n = _int(0)
    rc = lib().tv_device_count(ctypes.byref(n))
    if rc:
        raise NativeError(rc, _thread_error())
    return n.value


def cpu_share() -> int:
    """tv_cpu_share: the host CPUs this process may use as the library sees them (no GPU call)."""
    n = ctypes.c_uint32(0)
    rc = lib().tv_cpu_share(ctypes.byref(n))
    if rc:
        raise NativeError(rc, _thread_error())
    return n.value


def _thread_error() -> str:
    buf = ctypes.create_string_buffer(1024)
    lib().tv_last_error(None, buf, len(buf))
    return buf.value.decode(errors="replace")


class PinnedBuffer:
    """Page-locked host buffer (tv_host_alloc); exposes a writable memoryview `mv`."""

    def __init__(self, nbytes: int):
        self._L = lib()
        p = _p()
        rc = self._L.tv_host_alloc(nbytes, ctypes.byref(p))
        if rc:
            raise NativeError(rc, _thread_error())
        self.ptr = p.value
        self.nbytes = nbytes
        self.mv = memoryview((ctypes.c_char * nbytes).from_address(self.ptr)).cast("B") if nbytes else memoryview(b"")

    def close(self):
        if getattr(self, "ptr", None):
            self.mv.release()
            self._L.tv_host_free(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One GPU.  Thin RAII wrapper over tv_ctx*; every failing call raises NativeError."""

    def __init__(self, device: int = 0):
        self._L = lib()
        h = _p()
        rc = self._L.tv_create(ctypes.byref(h), device)
        if rc:
            raise NativeError(rc, _thread_error())
        self._h = h
        self.device = device
        self.shard_first = 0
        self.shard_count = 0
        self.thread_budget = 16   # host threads this context's call may use (verify._run_shards sets its share)

    # -- plumbing ----------------------------------------------------------------------
    def _err(self) -> str:
        buf = ctypes.create_string_buffer(1024)
        self._L.tv_last_error(self._h, buf, len(buf))
        return buf.value.decode(errors="replace")

    def _check(self, rc: int) -> None:
        if rc:
            raise NativeError(rc, self._err())

    def close(self) -> None:
        for b in getattr(self, "_batch_bufs", None) or ():   # verify_pieces' page-locked batch buffers
            b.close()
        self._batch_bufs = None
        if getattr(self, "_h", None):
            self._L.tv_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- API ---------------------------------------------------------------------------
    def set_option(self, key: int, value: int) -> None:
        self._check(self._L.tv_set_option(self._h, key, value))

    def get_option(self, key: int) -> int:
        v = _i64(0)
        self._check(self._L.tv_get_option(self._h, key, ctypes.byref(v)))
        return v.value

    def set_layout(self, total_length: int, piece_length: int, n_pieces: int,
                   shard_first: int = 0, shard_count: Optional[int] = None) -> None:
        if shard_count is None:
            shard_count = n_pieces - shard_first
        self._check(self._L.tv_set_layout(self._h, total_length, piece_length, n_pieces, shard_first, shard_count))
        self.shard_first, self.shard_count = shard_first, shard_count
        self.total_length, self.piece_length, self.n_pieces = total_length, piece_length, n_pieces

    def set_digests(self, pieces_raw: bytes) -> None:
        a, keep = _addr(pieces_raw)
        self._check(self._L.tv_set_digests(self._h, a, len(pieces_raw)))
        del keep

    def stage(self, linear_offset: int, data) -> None:
        a, keep = _addr(data)
        n = memoryview(data).nbytes
        self._check(self._L.tv_stage(self._h, linear_offset, a, n))
        del keep

    def stage_many(self, parts) -> None:
        """tv_stage_many: [(linear_offset, data), ...] staged in order in one call (no gather copy here)."""
        parts = list(parts)
        if not parts:
            return
        n = len(parts)
        offs, ptrs, lens = (ctypes.c_uint64 * n)(), (ctypes.c_uint64 * n)(), (ctypes.c_uint64 * n)()
        keeps = []
        for k, (off, data) in enumerate(parts):
            a, keep = _addr(data)
            keeps.append(keep)
            offs[k], ptrs[k], lens[k] = off, a or 0, memoryview(data).nbytes
        self._check(self._L.tv_stage_many(self._h, n, offs, ptrs, lens))
        del keeps

    def stage_ranges(self, buf, linear_offsets, buf_offsets, lens) -> None:
        """tv_stage_many over ranges of ONE host buffer: range k is buf[buf_offsets[k] : + lens[k]] staged at LINEAR
        linear_offsets[k] (e.g. a payload in memory and its file table: one range per file).  The addresses are
        computed with numpy (stage_many's per-buffer address lookup costs ~5 us in Python: 50 ms for 10,000 files)."""
        import numpy as np
        lo = np.ascontiguousarray(linear_offsets, dtype=np.uint64)
        bo = np.ascontiguousarray(buf_offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint64)
        n = len(lo)
        if n == 0:
            return
        if len(bo) != n or len(ln) != n:
            raise ValueError("stage_ranges: linear_offsets, buf_offsets and lens differ in length")
        base, keep = _addr(buf)
        size = memoryview(buf).nbytes
        # (checked without adding, so a huge offset -- e.g. a negative one cast to uint64 -- cannot wrap past it)
        sz = np.uint64(size)
        if bool((bo > sz).any()) or bool((ln > sz - np.minimum(bo, sz)).any()):
            raise ValueError("stage_ranges: a range reaches past the buffer")
        ptrs = bo + np.uint64(base or 0)
        self._check(self._L.tv_stage_many(self._h, n, lo.ctypes.data, ptrs.ctypes.data, ln.ctypes.data))
        del keep

    def stage_file(self, path, file_offset: int, linear_offset: int, length: int) -> bool:
        """tv_stage_file: stage `length` bytes of file `path` from `file_offset` as linear bytes
        [linear_offset, +length).  False when the file is missing, unopenable or short (TV_ERR_IO): the
        library then marks the pieces the reference's fsStorage.get would return null for (from the one
        holding the first missing byte on; tv_verify reports them 0 until the next set_layout)."""
        rc = self._L.tv_stage_file(self._h, os.fsencode(path), file_offset, linear_offset, length)
        if rc == TV_ERR_IO:
            return False
        self._check(rc)
        return True

    def stage_file_table(self, lengths, paths) -> list:
        """tv_stage_file_table: the shard's bytes from the torrent's file table (file k: lengths[k] bytes at
        paths[k], in info.files order); the library makes Storage.get's walk itself.  One status per FILE."""
        import numpy as np

        n = len(paths)
        if len(lengths) != n:
            raise ValueError("stage_file_table: lengths and paths differ in length")
        if n == 0:
            return []
        if all(type(x) is str for x in paths):
            blob = ("\0".join(paths) + "\0").encode(sys.getfilesystemencoding(), "surrogateescape")
        else:
            blob = b"\0".join(os.fsencode(x) for x in paths) + b"\0"
        if blob.count(b"\0") != n:
            raise ValueError("stage_file_table: a path contains a NUL byte")
        ln = np.ascontiguousarray(lengths, dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        self._check(self._L.tv_stage_file_table(self._h, n, ln.ctypes.data, blob, len(blob), st.ctypes.data))
        return st.tolist()

    def stream_file_table(self, lengths, paths, avail: Optional[bytes] = None) -> tuple:
        """tv_stream_file_table: the resume check from the files through the bounded ring (the library's readers
        fill each column's rows from the file table).  -> (bitfield, per-file statuses)."""
        import numpy as np

        n = len(paths)
        if len(lengths) != n:
            raise ValueError("stream_file_table: lengths and paths differ in length")
        if n and all(type(x) is str for x in paths):
            blob = ("\0".join(paths) + "\0").encode(sys.getfilesystemencoding(), "surrogateescape")
        else:
            blob = b"\0".join(os.fsencode(x) for x in paths) + b"\0" if n else b"\0"
        if n and blob.count(b"\0") != n:
            raise ValueError("stream_file_table: a path contains a NUL byte")
        ln = np.ascontiguousarray(lengths if n else [0], dtype=np.uint64)
        st = np.zeros(max(1, n), dtype=np.int32)
        out = ctypes.create_string_buffer(max(1, self._nbits()))
        a, keep = _addr(avail)
        self._check(self._L.tv_stream_file_table(self._h, n, ln.ctypes.data, blob, len(blob), a, out, st.ctypes.data))
        del keep
        return out.raw[: self._nbits()], st[:n].tolist()

    def stage_files(self, paths, file_offsets, linear_offsets, lens) -> list:
        """tv_stage_files: stage many file segments in one call.  Returns one status per segment:
        TV_OK, or TV_ERR_IO for a missing / unreadable / short file.  The library marks the pieces
        fsStorage.get would return null for itself (tv_verify reports them 0); the status is informational."""
        import numpy as np

        n = len(paths)
        if n == 0:
            return []
        if any(len(v) != n for v in (file_offsets, linear_offsets, lens)):
            raise ValueError("stage_files: paths, file_offsets, linear_offsets and lens differ in length")
        # all paths in one NUL-separated buffer (paths hold no NUL), and the char* array pointing into it;
        # str paths are encoded in one call (os.fsencode per path cost ~5 ms for 10,000 files)
        if all(type(x) is str for x in paths):
            blob = ("\0".join(paths) + "\0").encode(sys.getfilesystemencoding(), "surrogateescape")
        else:
            blob = b"\0".join(os.fsencode(x) for x in paths) + b"\0"
        if blob.count(b"\0") != n:
            raise ValueError("stage_files: a path contains a NUL byte")
        cblob = ctypes.create_string_buffer(blob, len(blob))
        nul = np.flatnonzero(np.frombuffer(blob, dtype=np.uint8) == 0)
        starts = np.empty(n, dtype=np.uint64)
        starts[0] = 0
        starts[1:] = nul[:-1] + 1
        ptrs = starts + np.uint64(ctypes.addressof(cblob))
        arr = lambda v: np.ascontiguousarray(v, dtype=np.uint64)  # noqa: E731
        fo, lo, ln = arr(file_offsets), arr(linear_offsets), arr(lens)
        st = np.zeros(n, dtype=np.int32)
        self._check(self._L.tv_stage_files(self._h, n, ptrs.ctypes.data, fo.ctypes.data, lo.ctypes.data,
                                           ln.ctypes.data, st.ctypes.data))
        del cblob
        return st.tolist()

    def read(self, linear_offset: int, out) -> None:
        """Copy resident bytes at linear_offset into the writable buffer `out` (tv_read)."""
        a, keep = _addr(out, writable=True)
        n = memoryview(out).nbytes
        self._check(self._L.tv_read(self._h, linear_offset, a, n))
        del keep

    def fill_synthetic(self, seed: int) -> None:
        self._check(self._L.tv_fill_synthetic(self._h, seed))

    def _nbits(self) -> int:
        return (self.shard_count + 7) // 8

    def verify(self, avail_bits=None) -> bytes:
        out = ctypes.create_string_buffer(max(1, self._nbits()))
        a, keep = _addr(avail_bits)
        self._check(self._L.tv_verify(self._h, a, out))
        del keep
        return out.raw[: self._nbits()]

    def verify_host(self, src, avail_bits=None) -> bytes:
        out = ctypes.create_string_buffer(max(1, self._nbits()))
        a, k1 = _addr(src)
        b, k2 = _addr(avail_bits)
        n = memoryview(src).nbytes if src is not None else 0
        self._check(self._L.tv_verify_host(self._h, a, n, b, out))
        del k1, k2
        return out.raw[: self._nbits()]

    def verify_list(self, pieces) -> bytes:
        """tv_verify_list: one byte (0/1) per listed global piece index."""
        n = len(pieces)
        if n == 0:
            return b""
        arr = (ctypes.c_uint64 * n)(*pieces)
        out = ctypes.create_string_buffer(n)
        self._check(self._L.tv_verify_list(self._h, ctypes.cast(arr, _p), n, out))
        return out.raw[:n]

    # -- streamed verify (tv_stream_*): bounded pinned ring, end-to-end resume check ----
    def stream_begin(self, avail_bits=None) -> None:
        a, keep = _addr(avail_bits)
        self._check(self._L.tv_stream_begin(self._h, a))
        del keep

    def stream_next(self) -> StreamReq:
        """The next request (req.rows == 0: every byte has been requested)."""
        req = StreamReq()
        self._check(self._L.tv_stream_next(self._h, ctypes.byref(req)))
        return req

    def row_bytes(self, req: StreamReq, q: int) -> int:
        """Valid bytes of row q: min(width, piece_len - offset) (piece.ts:16-19)."""
        i = req.piece + q
        L, P, total = self.piece_length, self.n_pieces, self.total_length
        plen = total % L if (i == P - 1 and total % L) else L
        return max(0, min(req.width, plen - req.offset))

    def stream_slot(self, req: StreamReq) -> memoryview:
        """Writable view of the request's pinned slot: row q at [q*width, q*width + row_bytes(q))."""
        n = req.rows * req.width
        return memoryview((ctypes.c_char * n).from_address(req.slot)).cast("B")

    def stream_commit(self, req: StreamReq) -> None:
        self._check(self._L.tv_stream_commit(self._h, ctypes.byref(req)))

    def stream_commit_from(self, req: StreamReq, src, pitch: int, src_offset: int = 0) -> None:
        """Rows from caller memory: row q at src[src_offset + q*pitch:][:row_bytes(q)] (bounds-checked)."""
        mv = memoryview(src).cast("B")
        need = 0   # end of the last row that has bytes (only the short last piece's row can have fewer)
        for q in (req.rows - 1, req.rows - 2):
            if q >= 0 and self.row_bytes(req, q):
                need = src_offset + q * pitch + self.row_bytes(req, q)
                break
        if need > mv.nbytes or src_offset < 0:
            raise ValueError(f"stream_commit_from: the rows need {need} bytes of src, it has {mv.nbytes}")
        a, keep = _addr(src)
        self._check(self._L.tv_stream_commit_from(self._h, ctypes.byref(req), (a or 0) + src_offset, pitch))
        del keep

    def stream_unreadable(self, piece: int) -> None:
        self._check(self._L.tv_stream_unreadable(self._h, piece))

    def stream_fill_synthetic(self, req: StreamReq, seed: int) -> None:
        self._check(self._L.tv_stream_fill_synthetic(self._h, ctypes.byref(req), seed))

    def stream_end(self) -> bytes:
        out = ctypes.create_string_buffer(max(1, self._nbits()))
        self._check(self._L.tv_stream_end(self._h, out))
        return out.raw[: self._nbits()]

    def stream_abort(self) -> None:
        self._check(self._L.tv_stream_abort(self._h))

    def hash(self) -> bytes:
        out = ctypes.create_string_buffer(max(1, 20 * self.shard_count))
        self._check(self._L.tv_hash(self._h, out))
        return out.raw[: 20 * self.shard_count]

    def last_timing(self) -> tuple:
        k, t = ctypes.c_double(0), ctypes.c_double(0)
        self._check(self._L.tv_last_timing(self._h, ctypes.byref(k), ctypes.byref(t)))
        return k.value, t.value

    def last_kernel(self) -> tuple:
        k, n = _int(0), _int(0)
        self._check(self._L.tv_last_kernel(self._h, ctypes.byref(k), ctypes.byref(n)))
        return k.value, n.value

    def counter(self, key: int) -> int:
        """tv_get_counter: device allocations since creation / bytes held now (TV_COUNTER_*)."""
        v = _u64(0)
        self._check(self._L.tv_get_counter(self._h, key, ctypes.byref(v)))
        return v.value

    def synchronize(self) -> None:
        self._check(self._L.tv_synchronize(self._h))

    def set_companions(self, on: bool) -> None:
        """TV_OPT_TWIN_FILL: light companion workgroups on the idle SIMDs of twin launches with fewer than 2 workgroups
        per CU (default: on, unless other processes hold >= 1 GiB of the GPU's memory); False keeps them off
        whatever the GPU's other users.  The bitfields are the same either way."""
        self.set_option(TV_OPT_TWIN_FILL, 1 if on else 0)

    def set_clock_probe(self, on: bool) -> None:
        """TV_OPT_CLOCK_PROBE: verify / hash launches record the shader clock they ran at (last_clock_khz)."""
        self.set_option(TV_OPT_CLOCK_PROBE, 1 if on else 0)

    def last_clock_khz(self) -> int:
        """The shader clock of the last probed launch's workgroup 0, kHz (0: no probe); waits for the compute stream."""
        return self.counter(TV_COUNTER_LAST_CLOCK_KHZ)

    def _reset_file_clock(self) -> None:
        """Zero the file-staging phase clock (internal: TV_OPT_FILE_CLOCK_RESET)."""
        self.set_option(TV_OPT_FILE_CLOCK_RESET, 1)

    def _file_clock(self) -> dict:
        """The file-staging phase clock since the last reset: {phase: ns (or bytes for bytes_*)} (internal counters
        TV_COUNTER_FILE_CLOCK + TV_FILE_PHASE_*, tv_options_internal.h)."""
        return {ph: self.counter(TV_COUNTER_FILE_CLOCK + k) for k, ph in enumerate(TV_FILE_PHASES)}
