"""Page-cache helpers for the file-backed benches (tools/f2_stamps.py, tools/storage_paths_bench.py).

resident(paths)   -> fraction of the files' pages in the page cache (mmap + mincore per file, summed by pages)
drop_cache(paths) -> fsync + posix_fadvise(DONTNEED) on every file, repeated until <= max_resident of the pages are
                     still cached (or `tries` passes), returning the residency it reached.  A "cold" measurement
                     whose files are still cached measures the page cache, not the disk, so the
                     benches record this figure in every cold line and refuse to call a leg cold above 1 %.
"""
import ctypes
import ctypes.util
import mmap
import os
import time

import numpy as np

_libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
_libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
_libc.mincore.restype = ctypes.c_int
_PAGE = os.sysconf("SC_PAGE_SIZE")


_libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
_libc.mmap.restype = ctypes.c_void_p
_libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
_MAP_FAILED = ctypes.c_void_p(-1).value


def _file_pages(path):
    """(pages resident, pages) of one file: a read-only shared mapping of it, mincore, unmapped."""
    n = os.path.getsize(path)
    if n == 0:
        return 0, 0
    fd = os.open(path, os.O_RDONLY)
    try:
        addr = _libc.mmap(None, n, mmap.PROT_READ, mmap.MAP_SHARED, fd, 0)
        if addr in (None, _MAP_FAILED):
            raise OSError(ctypes.get_errno(), "mmap " + path)
        try:
            npages = (n + _PAGE - 1) // _PAGE
            vec = (ctypes.c_ubyte * npages)()
            if _libc.mincore(addr, n, vec) != 0:
                raise OSError(ctypes.get_errno(), "mincore " + path)
            return int((np.frombuffer(vec, np.uint8) & 1).sum()), npages
        finally:
            _libc.munmap(addr, n)
    finally:
        os.close(fd)


def resident(paths):
    """Fraction of the pages of `paths` that are in the page cache."""
    have = total = 0
    for p in paths:
        h, t = _file_pages(p)
        have += h
        total += t
    return have / total if total else 0.0


def drop_cache(paths, max_resident=0.01, tries=3):
    """Evict the files from the page cache (no root needed: fsync, then POSIX_FADV_DONTNEED); the residency left."""
    r = 1.0
    for _ in range(tries):
        for p in paths:
            fd = os.open(p, os.O_RDONLY)
            try:
                os.fsync(fd)
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            finally:
                os.close(fd)
        r = resident(paths)
        if r <= max_resident:
            break
        time.sleep(0.5)     # dirty pages still under writeback are not dropped: let it finish
    return r


def fs_type(path):
    """The filesystem type of the mount holding `path` (/proc/mounts, longest matching mount point)."""
    path = os.path.realpath(path)
    best, kind = "", "unknown"
    try:
        for line in open("/proc/mounts"):
            parts = line.split()
            mnt = parts[1].replace("\\040", " ")
            if (path == mnt or path.startswith(mnt.rstrip("/") + "/")) and len(mnt) > len(best):
                best, kind = mnt, parts[2]
    except OSError:
        pass
    return kind


def evictable(d, mib=64):
    """Can files under directory `d` be made cold (DONTNEED drops them)?  -> dict(dir, fs, ok, resident_after)."""
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, f".evict_probe_{os.getpid()}")
    try:
        with open(p, "wb") as f:
            f.write(os.urandom(1 << 20) * mib)
        r = drop_cache([p])
        return {"dir": d, "fs": fs_type(d), "ok": r <= 0.01, "resident_after_drop": round(r, 4)}
    except OSError as exc:
        return {"dir": d, "fs": fs_type(d), "ok": False, "error": str(exc)}
    finally:
        try:
            os.unlink(p)
        except OSError:
            pass


if __name__ == "__main__":
    import json
    import sys
    if len(sys.argv) > 2 and sys.argv[1] == "pick":
        # print the first directory whose files can be evicted (else the first one given), details on stderr
        probes = [evictable(d) for d in sys.argv[2:] if d]
        print(json.dumps(probes), file=sys.stderr)
        good = [x["dir"] for x in probes if x["ok"]]
        print(good[0] if good else sys.argv[2])
