"""Storage plugin API and the file-to-piece mapping, mirroring reference storage.ts.

* StorageMethod {get, set, exists} is the reference's only plugin API (storage.ts:16-26).
* Storage maps the linear torrent byte space to files (storage.ts:41-137).
  `segments(offset, length)` is `findAndDo`'s walk (storage.ts:89-137) returned as data:
  ordered (path, file_offset, n_bytes, slice_start) tuples.  It keeps the reference's
  quirks: single-file paths are [*dir, name] (:99-101); multi-file paths are
  [*dir, *file.path] WITHOUT info.name (:114); `fileEnd >= offset` emits a zero-length
  segment at an exact file boundary (:109-110); a range past the last file fails (:136).
* Any action failure or exception makes get() return None and set() return False
  (storage.ts:130-136, 163-171).
* fs_storage opens with read/write/create like OPEN_OPTIONS (storage.ts:28-32), so get() on
  a missing file creates it empty and then fails the read -> None (storage_test.ts:59-62).

The same segment walk produces the device offset table for multi-file torrents: the GPU
path stages each segment at its linear offset, so pieces spanning file boundaries are
contiguous in HBM (see verify.py).
"""
from __future__ import annotations

import bisect
import ctypes
import os
from typing import Callable, List, Optional, Protocol, Tuple

from .piece import BLOCK_SIZE

Segment = Tuple[List[str], int, int, int]  # (path, file_offset, n_bytes, slice_start)


class StorageMethod(Protocol):
    def get(self, path: List[str], offset: int, length: int) -> Optional[bytes]: ...

    def set(self, path: List[str], offset: int, data: bytes) -> bool: ...

    def exists(self, path: List[str]) -> bool: ...


def _split_dir(dir_path: str) -> List[str]:
    # storage.ts:45-48: relative(Deno.cwd(), dirPath).split(SEP), leading "" dropped
    rel = os.path.relpath(dir_path, os.getcwd())
    parts = rel.split(os.sep)
    if rel == ".":
        parts = [""]
    if parts and parts[0] == "":
        parts = parts[1:]
    return parts


class Storage:
    """storage.ts:34-138."""

    def __init__(self, method: StorageMethod, info, dir_path: str):
        self.method = method
        self.info = info
        self.dir_path = _split_dir(dir_path)
        self._written: dict = {}
        self._ends: Optional[List[int]] = None  # cumulative file ends (lazy)
        self._table = None                       # (starts, ends) as int64 arrays (lazy)
        self._joined: Optional[List[str]] = None  # os.path.join of every file's path (lazy)

    # -- mapping ---------------------------------------------------------------------
    def segments(self, offset: int, length: int) -> Optional[List[Segment]]:
        """findAndDo's walk (storage.ts:89-137) without the action.  None = unmappable."""
        if self.info.files is None:
            return [([*self.dir_path, self.info.name], offset, length, 0)]
        if self._ends is None:
            ends, acc = [], 0
            for f in self.info.files:
                acc += f.length
                ends.append(acc)
            self._ends = ends
        ends = self._ends
        # the reference walks every file from the first (storage.ts:105-128) and acts on the first
        # file whose end is >= offset; files before it do nothing, so start there (bisect).
        k = bisect.bisect_left(ends, offset)
        out: List[Segment] = []
        i = 0
        file_start = ends[k - 1] if k > 0 else 0
        files = self.info.files
        for idx in range(k, len(files)):
            f = files[idx]
            file_end = file_start + f.length
            if file_end >= offset:
                n_bytes = min(file_end - offset - i, length - i)
                file_offset = max(0, offset - file_start)
                out.append(([*self.dir_path, *f.path], file_offset, n_bytes, i))
                i += n_bytes
                if i == length:
                    return out
            file_start = file_end
        return None

    def segment_arrays(self, offset: int, length: int):
        """segments(offset, length) without its zero-length entries, as arrays: (file_index,
        file_offset, n_bytes, slice_start), int64 each, in walk order; file_index is into info.files
        (all 0 for a single-file torrent).  None = unmappable, exactly when segments() returns None.

        The same walk, vectorised for many-file shards: the file k that segments() visits contributes
        the bytes [max(start_k, offset), min(end_k, offset + length)), so every file overlapping the
        range gives one segment, and the walk completes iff the files reach offset + length."""
        import numpy as np

        if self.info.files is None:
            n = length if length > 0 else 0
            if n == 0:
                return tuple(np.zeros(0, np.int64) for _ in range(4))
            return (np.zeros(1, np.int64), np.array([offset], np.int64), np.array([n], np.int64),
                    np.zeros(1, np.int64))
        if self._table is None:
            lens = np.fromiter((f.length for f in self.info.files), dtype=np.int64, count=len(self.info.files))
            ends = np.cumsum(lens)
            self._table = (ends - lens, ends)
        starts, ends = self._table
        if len(ends) == 0 or int(ends[-1]) < offset + length:
            return None
        a = int(np.searchsorted(ends, offset, side="right"))           # first file ending past offset
        b = int(np.searchsorted(starts, offset + length, side="left"))  # files starting before the end
        k = np.arange(a, max(a, b), dtype=np.int64)
        lo = np.maximum(starts[a:b], offset)
        n = np.minimum(ends[a:b], offset + length) - lo
        keep = n > 0
        k, lo, n = k[keep], lo[keep], n[keep]
        return k, lo - starts[k], n, lo - offset

    def zero_length_segments(self, offset: int, length: int, piece_length: int):
        """The zero-length segments of the walks Storage.get makes for the pieces tiling [offset, offset +
        length) (offset a multiple of piece_length), as arrays (file_index, file_offset, linear_offset).
        findAndDo (storage.ts:105-128) emits one for every file whose end e lies inside the piece's range
        [o, o + n) and that contributes nothing there: a file ending exactly where the piece starts (e == o,
        `fileEnd >= offset`, :109-110) or a zero-length file inside the piece.  Their piece is
        linear_offset // piece_length.  fsStorage.get still opens such a path (storage.ts:158), so its
        open decides whether the piece is null (tv_stage_files checks it)."""
        import numpy as np

        if self.info.files is None or length <= 0:
            return tuple(np.zeros(0, np.int64) for _ in range(3))
        if self._table is None:
            lens = np.fromiter((f.length for f in self.info.files), dtype=np.int64, count=len(self.info.files))
            ends = np.cumsum(lens)
            self._table = (ends - lens, ends)
        starts, ends = self._table
        lens = ends - starts
        a = int(np.searchsorted(ends, offset, side="left"))
        b = int(np.searchsorted(ends, offset + length, side="left"))
        k = np.arange(a, b, dtype=np.int64)
        e = ends[a:b]
        keep = (lens[a:b] == 0) | (e % piece_length == 0)
        k, e = k[keep], e[keep]
        return k, lens[k], e

    def file_paths(self) -> List[str]:
        """os.path.join(*segment path) for every file index of segment_arrays (fs_storage's paths)."""
        if self._joined is None:
            if self.info.files is None:
                self._joined = [os.path.join(*self.dir_path, self.info.name)]
            else:
                base = os.path.join(*self.dir_path) if self.dir_path else ""
                head = base if (not base or base.endswith(os.sep)) else base + os.sep
                sep, dsep = os.sep, os.sep + os.sep
                out = []
                for f in self.info.files:
                    # os.path.join(*dir, *parts) without its per-call cost: the plain join equals it exactly
                    # when no part is empty or absolute, i.e. when the joined string neither starts nor ends
                    # with the separator and holds no doubled separator
                    j = sep.join(f.path)
                    if j and j[0] != sep and j[-1] != sep and dsep not in j:
                        out.append(head + j)
                    else:
                        out.append(os.path.join(*self.dir_path, *f.path))
                self._joined = out
        return self._joined

    def _find_and_do(self, offset: int, buf: bytearray | memoryview,
                     action: Callable[[List[str], int, memoryview], bool]) -> bool:
        try:
            segs = self.segments(offset, len(buf))
            if segs is None:
                return False
            mv = memoryview(buf)
            for path, foff, n, start in segs:
                if not action(path, foff, mv[start:start + n]):
                    return False
            return True
        except Exception:
            return False

    # -- reference API -----------------------------------------------------------------
    def get(self, offset: int, length: int):
        """storage.ts:50-65: the bytes [offset, offset + length) read file segment by file segment through
        the method, or None when a segment fails.  A segment the method returns SHORTER than asked fills the
        front of its slice and leaves the rest zero, as the reference's slice.set(got) into its zeroed
        Uint8Array does (:51,57-58); a LONGER one makes the whole get null (slice.set throws a RangeError,
        which findAndDo's catch turns into false, :130-133).  A range inside one file is the method's own bytes
        when they have the full length (no copy); the segments of a range spanning files are copied into one
        buffer with the GIL released (memmove), so many readers copy in parallel."""
        try:
            segs = self.segments(offset, length)
            if segs is None:
                return None
            if len(segs) == 1:
                path, foff, n, _ = segs[0]
                got = self.method.get(path, foff, n)
                if got is None or len(got) > n:
                    return None
                if len(got) == n:
                    return got
                out = bytearray(n)
                out[:len(got)] = got
                return out
            out = bytearray(length)
            base = ctypes.addressof((ctypes.c_char * length).from_buffer(out)) if length else 0
            for path, foff, n, start in segs:
                got = self.method.get(path, foff, n)
                if got is None or len(got) > n:
                    return None
                if len(got):
                    copy_bytes(base + start, got, len(got))
            return out
        except Exception:
            return None

    def set(self, offset: int, data: bytes) -> bool:
        """storage.ts:67-87 (blocks deduplicated by offset / BLOCK_SIZE)."""
        index = offset / BLOCK_SIZE
        if self._written.get(index):
            return True
        ok = self._find_and_do(offset, bytearray(data),
                               lambda path, foff, sl: self.method.set(path, foff, bytes(sl)))
        if ok:
            self._written[index] = True
        return ok


def copy_bytes(dst: int, src, n: int) -> None:
    """memmove n bytes of the bytes-like `src` to address dst, without the GIL (ctypes' C call) and without a
    temporary copy of src."""
    if isinstance(src, bytes):
        ctypes.memmove(dst, src, n)                      # (a bytes argument is passed by its own address)
        return
    mv = memoryview(src).cast("B")
    if mv.readonly:
        ctypes.memmove(dst, bytes(mv[:n]), n)
    else:
        ctypes.memmove(dst, (ctypes.c_char * mv.nbytes).from_buffer(mv), n)


class FsStorage:
    """fsStorage (storage.ts:149-206)."""

    def get(self, path: List[str], offset: int, length: int) -> Optional[bytes]:
        p = os.path.join(*path)
        try:
            fd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
        except OSError:
            return None
        try:
            data = os.pread(fd, length, offset) if length else b""
            if len(data) != length:  # readN: UnexpectedEof (_bytes.ts:13-17)
                return None
            return data
        except OSError:
            return None
        finally:
            os.close(fd)

    def set(self, path: List[str], offset: int, data: bytes) -> bool:
        p = os.path.join(*path)
        try:
            try:
                fd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
            except FileNotFoundError:
                os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
                fd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
            try:
                view = memoryview(data)
                while view:
                    n = os.pwrite(fd, view, offset)
                    view = view[n:]
                    offset += n
            finally:
                os.close(fd)
            return True
        except OSError:
            return False

    def exists(self, path: List[str]) -> bool:
        return os.path.exists(os.path.join(*path))


fs_storage = FsStorage()


class MemoryStorage:
    """An in-memory StorageMethod (tests / synthetic torrents): path tuple -> bytearray.
    Missing path or a read past the end -> None, like fsStorage's EOF."""

    def __init__(self, files: Optional[dict] = None):
        self.files = {tuple(k): bytearray(v) for k, v in (files or {}).items()}

    def get(self, path, offset, length):
        f = self.files.get(tuple(path))
        if f is None:
            return None if length else b""
        if offset + length > len(f):
            return None
        return bytes(f[offset:offset + length])

    def set(self, path, offset, data):
        f = self.files.setdefault(tuple(path), bytearray())
        if len(f) < offset + len(data):
            f.extend(b"\0" * (offset + len(data) - len(f)))
        f[offset:offset + len(data)] = data
        return True

    def exists(self, path):
        return tuple(path) in self.files
