"""ctypes binding of libtorrent_verify.so (include/torrent_verify.h).

This is the Python analogue of the Deno `Deno.dlopen` binding in ts/verify.ts: the same
symbols, the same argument meaning, negative status -> exception.  There is no CPU fallback:
if the library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TORRENT_VERIFY_LIB", os.path.join(_PKG, "libtorrent_verify.so"))

TV_OK = 0
TV_ERR_ARG = -1
TV_ERR_HIP = -2
TV_ERR_STATE = -3
TV_ERR_NOMEM = -4
TV_ERR_IO = -5

TV_OPT_KERNEL = 1
TV_OPT_STRIDE_PAD = 2
TV_OPT_STREAM_CHUNK = 3
TV_OPT_SPLIT_PAIRS = 4
TV_OPT_FILE_DIRECT = 5
TV_OPT_FILE_CHUNK = 6
TV_OPT_FILE_DIRECT_MIN = 7
TV_OPT_FILE_THREADS = 8
TV_OPT_FILE_CONCURRENT = 9

KERNEL_AUTO, KERNEL_LANE, KERNEL_SPLIT = 0, 1, 2

# every symbol include/torrent_verify.h declares: (name, restype, argtypes)
_u64, _i64, _int, _p = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
SYMBOLS = [
    ("tv_abi_version", _int, []),
    ("tv_device_count", _int, [ctypes.POINTER(_int)]),
    ("tv_create", _int, [ctypes.POINTER(_p), _int]),
    ("tv_destroy", None, [_p]),
    ("tv_last_error", _int, [_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("tv_set_layout", _int, [_p, _u64, _u64, _u64, _u64, _u64]),
    ("tv_set_digests", _int, [_p, _p, _u64]),
    ("tv_stage", _int, [_p, _u64, _p, _u64]),
    ("tv_stage_file", _int, [_p, ctypes.c_char_p, _u64, _u64, _u64]),
    ("tv_stage_files", _int, [_p, _u64, _p, _p, _p, _p, _p]),
    ("tv_read", _int, [_p, _u64, _p, _u64]),
    ("tv_fill_synthetic", _int, [_p, _u64]),
    ("tv_verify", _int, [_p, _p, _p]),
    ("tv_verify_host", _int, [_p, _p, _u64, _p, _p]),
    ("tv_verify_list", _int, [_p, _p, _u64, _p]),
    ("tv_hash", _int, [_p, _p]),
    ("tv_set_option", _int, [_p, _int, _i64]),
    ("tv_get_option", _int, [_p, _int, ctypes.POINTER(_i64)]),
    ("tv_last_timing", _int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    ("tv_last_kernel", _int, [_p, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
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


def _addr(buf) -> tuple:
    """(void* address, keepalive) of a bytes-like object or None."""
    if buf is None:
        return None, None
    if isinstance(buf, bytes):
        return ctypes.cast(ctypes.c_char_p(buf), _p).value, buf
    mv = memoryview(buf).cast("B")
    if mv.nbytes == 0:
        return None, None
    if mv.readonly:
        b = bytes(mv)
        return ctypes.cast(ctypes.c_char_p(b), _p).value, b
    c = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return ctypes.addressof(c), c


def device_count() -> int:
    n = _int(0)
    rc = lib().tv_device_count(ctypes.byref(n))
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

    # -- plumbing ----------------------------------------------------------------------
    def _err(self) -> str:
        buf = ctypes.create_string_buffer(1024)
        self._L.tv_last_error(self._h, buf, len(buf))
        return buf.value.decode(errors="replace")

    def _check(self, rc: int) -> None:
        if rc:
            raise NativeError(rc, self._err())

    def close(self) -> None:
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

    def set_digests(self, pieces_raw: bytes) -> None:
        a, keep = _addr(pieces_raw)
        self._check(self._L.tv_set_digests(self._h, a, len(pieces_raw)))
        del keep

    def stage(self, linear_offset: int, data) -> None:
        a, keep = _addr(data)
        n = memoryview(data).nbytes
        self._check(self._L.tv_stage(self._h, linear_offset, a, n))
        del keep

    def stage_file(self, path, file_offset: int, linear_offset: int, length: int) -> bool:
        """tv_stage_file: stage `length` bytes of file `path` from `file_offset` as linear bytes
        [linear_offset, +length).  False when the file is missing or short (TV_ERR_IO: the
        reference's fsStorage.get -> null, so the pieces it touches are unreadable)."""
        rc = self._L.tv_stage_file(self._h, os.fsencode(path), file_offset, linear_offset, length)
        if rc == TV_ERR_IO:
            return False
        self._check(rc)
        return True

    def stage_files(self, paths, file_offsets, linear_offsets, lens) -> list:
        """tv_stage_files: stage many file segments in one call.  Returns one status per segment:
        TV_OK, or TV_ERR_IO for a missing / unreadable / short file (its pieces are unreadable)."""
        import numpy as np

        n = len(paths)
        if n == 0:
            return []
        if any(len(v) != n for v in (file_offsets, linear_offsets, lens)):
            raise ValueError("stage_files: paths, file_offsets, linear_offsets and lens differ in length")
        # all paths in one NUL-separated buffer (paths hold no NUL), and the char* array pointing into it
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
        a, keep = _addr(out)
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

    def synchronize(self) -> None:
        self._check(self._L.tv_synchronize(self._h))
