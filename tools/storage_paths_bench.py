"""The reference-shaped Storage paths against verify_files, warm and cold.

Layouts written under <dir> (payload: the splitmix64 generator, tests/synth.py's numpy form; digests: hashlib, 1 % of
them corrupted, so every result is checked against hashlib's bitfield):
  cfg3      BASELINE config 3: 10,000 files of U[0, 512 KiB], 256 KiB pieces (tests/layouts.py; committed bits)
  single16  one 16 GiB file, 1 MiB pieces (cfg2's geometry)
  files64   16 GiB in 64 files, 1 MiB pieces (the round-1 resume-from-disk layout)

Paths timed (each reads the files exactly as the reference would: Storage(fs_storage) = storage.ts's Storage over
fsStorage, which opens the file once per get call, storage.ts:149-172):
  verify_files                     one tv_stage_files call per shard (library readers / page-cache DMA)
  verify_pieces(Storage(fs))       one Storage.get per piece (default reader threads), double-buffered batches to HBM
  verify_stream(Storage(fs).get)   the bounded ring, whole-piece rows (TV_OPT_STREAM_ROWS, the default)
  verify_stream(..., chunk=L/4)    the bounded ring, columns: four gets per piece (the round-3 default)
Warm = the files were just written (page cache); cold = posix_fadvise(DONTNEED) after fsync on every file
(no root needed), re-checked with mincore (tools/fsutil.py): every line carries `resident`, the fraction of the
files' pages cached when the leg started, and a cold pass whose drop leaves more than 1 % cached is refused
(freshly written files on some boxes stayed cached and the "cold" legs read memory).  `read_ceiling` = the files read cold by 16 threads of 4 MiB preads into
host memory, nothing else: what the box's storage delivers.  Each line: GB/s, gets (= opens) per piece.

usage: python tools/storage_paths_bench.py <dir> [layout ...] > out.jsonl
"""
import copy
import itertools
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fsutil  # noqa: E402
from tests import synth  # noqa: E402  (the generator and hashlib digests: nothing under oracle/ runs here)
from torrent_amd import FileInfo, Storage, make_info, verify_files, verify_pieces, verify_stream  # noqa: E402
from torrent_amd.storage import FsStorage  # noqa: E402

MiB, GiB = 1 << 20, 1 << 30
COLD_MAX_RESIDENT = 0.01     # a leg is "cold" only with <= 1 % of its files' pages cached at its start


class CountingFs(FsStorage):
    """fsStorage with a count of get calls (each one an open, storage.ts:158)."""

    def __init__(self):
        self.reset()

    def reset(self) -> None:
        self._n = itertools.count()      # (next() on it is atomic under the GIL: no lock on the hot path)

    @property
    def gets(self) -> int:
        return next(copy.copy(self._n))  # (the count so far, without consuming it)

    def get(self, path, offset, length):
        next(self._n)
        return super().get(path, offset, length)


def emit(rec):
    print(json.dumps(rec), flush=True)


def drop_cache(paths):
    """Evict the files (fsutil.drop_cache: fsync + DONTNEED, re-checked with mincore); the residency left."""
    return fsutil.drop_cache(paths)


_RC_BIN = None


def _read_ceiling_bin():
    """tools/read_ceiling.c built with gcc into TMPDIR (once); None when it cannot be built."""
    global _RC_BIN
    if _RC_BIN is None:
        import subprocess
        import tempfile
        exe = os.path.join(tempfile.gettempdir(), f"read_ceiling_{os.getpid()}")
        try:
            subprocess.check_call(["gcc", "-O2", "-pthread", os.path.join(ROOT, "tools", "read_ceiling.c"), "-o", exe,
                                   "-ldl"])
            _RC_BIN = exe
        except (OSError, subprocess.CalledProcessError):
            _RC_BIN = ""
    return _RC_BIN or None


def read_ceiling(paths, threads=16, part=4 * MiB, direct=False, env=None):
    """Bytes/s of reading every file with `threads` parallel preads of `part` bytes (nothing kept): the C reader
    tools/read_ceiling.c (no GIL in the way: the Python form under-measured 10,000 small files), else Python."""
    exe = _read_ceiling_bin()
    if exe:
        import subprocess
        r = subprocess.run([exe, str(threads), str(part)] + (["direct"] if direct else []), input="\n".join(paths),
                           capture_output=True, text=True, check=True, env={**os.environ, **(env or {})})
        rec = json.loads(r.stdout)
        return rec["bytes"] / rec["seconds"]
    if direct:
        return None
    jobs = []
    for p in paths:
        n = os.path.getsize(p)
        jobs += [(p, o, min(part, n - o)) for o in range(0, n, part)]
    local = threading.local()

    def one(j):
        p, o, n = j
        fd = os.open(p, os.O_RDONLY)
        try:
            buf = getattr(local, "buf", None)
            if buf is None or len(buf) < part:
                buf = local.buf = bytearray(part)
            return os.preadv(fd, [memoryview(buf)[:n]], o)
        finally:
            os.close(fd)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(one, jobs))
    return total / (time.perf_counter() - t0)


def _buffered(fn):
    """fn() with the cached context's cold reads buffered (TV_OPT_FILE_ODIRECT = 0), then back to the default."""
    from torrent_amd import _native
    from torrent_amd.verify import _context
    with _context(0) as ctx:
        ctx.set_option(_native.TV_OPT_FILE_ODIRECT, 0)
    try:
        return fn()
    finally:
        with _context(0) as ctx:
            ctx.set_option(_native.TV_OPT_FILE_ODIRECT, 1)


def write_layout(name, d):
    """-> (info, expected bitfield bytes, file paths)."""
    os.makedirs(d, exist_ok=True)
    if name == "cfg3":
        from tests.layouts import build_layout, by_name
        lay = build_layout(by_name("cfg3"), fill=synth.fill)
        rec = {r["name"]: r for r in json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))}["cfg3"]
        paths = []
        for path, data in lay["disk_files"]().items():
            p = os.path.join(d, *path)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "wb") as f:
                f.write(data)
            paths.append(p)
        return lay["info"], bytes.fromhex(rec["expected_bitfield"]), paths
    L, total = MiB, 16 * GiB
    P = total // L
    nf = 1 if name == "single16" else 64
    seed = 16 if nf == 1 else 64
    digests = bytearray(synth.piece_digests(seed, total, L, P, threads=16))
    for i in range(5, P, 100):
        digests[20 * i + 3] ^= 0x08
    bits = bytearray(b"\xff" * (P // 8))     # hashlib digests of the written payload, 1 % corrupted
    for i in range(5, P, 100):
        bits[i >> 3] &= ~(0x80 >> (i & 7)) & 0xFF
    expect = bytes(bits)
    per = total // nf
    if nf == 1:
        files, paths = None, [os.path.join(d, "single16.bin")]
        sizes = [total]
    else:
        sizes = [per] * nf
        files = [FileInfo(s, [f"f{k:03d}.bin"]) for k, s in enumerate(sizes)]
        paths = [os.path.join(d, f"f{k:03d}.bin") for k in range(nf)]
    off = 0
    chunk = 256 * MiB
    for p, s in zip(paths, sizes):
        with open(p, "wb") as f:
            for o in range(0, s, chunk):
                n = min(chunk, s - o)
                f.write(synth.fill(seed, off + o, n))
        off += s
    info = make_info(L, bytes(digests), "single16.bin" if nf == 1 else "files64", files=files, length=total)
    return info, expect, paths


def timed(fn, reps):
    best, out = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return best, out


def main():
    d = sys.argv[1]
    names = sys.argv[2:] or ["cfg3", "single16", "files64"]
    st = os.statvfs(d if os.path.exists(d) else os.path.dirname(d.rstrip("/")) or "/")
    emit({"host": {"cpus_allowed": len(os.sched_getaffinity(0)), "free_disk_gib": round(st.f_bavail * st.f_frsize / GiB, 1)}})
    for name in names:
        root = os.path.join(d, name)
        t0 = time.perf_counter()
        info, expect, paths = write_layout(name, root)
        P, L, total = info.n_pieces, info.piece_length, info.length
        emit({"layout": name, "files": len(paths), "bytes": total, "pieces": P, "piece_length": L,
              "write_s": round(time.perf_counter() - t0, 1)})
        cwd = os.getcwd()
        os.chdir(root)           # Storage(fs_storage) paths are relative to the working directory (storage.ts)
        try:
            for cold in (False, True):
                legs = [("verify_files", lambda: verify_files(info, root), None)]
                if cold:   # the A/B of the cold reads: O_DIRECT (the default) against the page cache's reads
                    legs.append(("verify_files, buffered reads (TV_OPT_FILE_ODIRECT=0)", lambda: _buffered(
                        lambda: verify_files(info, root)), None))
                fs = CountingFs()
                st_ = Storage(fs, info, root)
                legs.append(("verify_pieces(Storage(fs))", lambda: verify_pieces(info, st_), fs))
                fs2 = CountingFs()
                st2 = Storage(fs2, info, root)
                legs.append(("verify_stream(Storage(fs).get) rows", lambda: verify_stream(info, st2.get), fs2))
                fs3 = CountingFs()
                st3 = Storage(fs3, info, root)
                legs.append((f"verify_stream(Storage(fs).get) columns chunk={L // 4}",
                             lambda: verify_stream(info, st3.get, chunk=L // 4), fs3))
                # the bound of the Storage paths: the gets alone (Storage(fs).get of every piece on the same reader
                # threads as verify_pieces, in the same runs of pieces; bytes dropped; no GPU)
                fs4 = CountingFs()
                st4 = Storage(fs4, info, root)
                from torrent_amd.piece import piece_length as _plen
                from torrent_amd.verify import _STORAGE_THREADS, _chunked_map

                def gets_only(threads=_STORAGE_THREADS):
                    with ThreadPoolExecutor(threads) as ex:
                        return sum(_chunked_map(ex, lambda i: st4.get(i * L, _plen(i, info)) is not None, P, threads))
                res = drop_cache(paths) if cold else fsutil.resident(paths)
                if cold and res > COLD_MAX_RESIDENT:
                    emit({"layout": name, "cache": "cold", "refused": True, "resident_after_drop": round(res, 4),
                          "why": "the page cache kept the files after fsync + POSIX_FADV_DONTNEED (e.g. a tmpfs or "
                                 "overlay directory): a 'cold' leg here would measure memory, not the disk"})
                    break
                el, n_ok = timed(gets_only, 1 if cold else 2)
                ngets = fs4.gets
                emit({"layout": name, "cache": "cold" if cold else "warm", "resident": round(res, 4),
                      "path": f"Storage(fs).get only, {_STORAGE_THREADS} threads",
                      "best_s": round(el, 3), "gbps": round(total / el / 1e9, 2), "us_per_get":
                      round(el / max(1, ngets / (1 if cold else 2)) * 1e6, 1),
                      "gets_per_piece": round(ngets / (1 if cold else 2) / P, 3)})
                if cold:
                    res = drop_cache(paths)
                    ceil = read_ceiling(paths)
                    emit({"layout": name, "cache": "cold", "read_ceiling_gbps": round(ceil / 1e9, 2),
                          "resident": round(res, 4),
                          "how": "tools/read_ceiling.c: 16 threads x 4 MiB preads of every file after the drop"})
                    res = drop_cache(paths)
                    try:
                        dceil = read_ceiling(paths, direct=True)
                    except Exception as exc:   # (a filesystem without O_DIRECT)
                        dceil, why = None, str(exc)[:200]
                    emit({"layout": name, "cache": "cold", "read_ceiling_direct_gbps": round(dceil / 1e9, 2) if dceil
                          else None, "resident": round(res, 4),
                          "how": "tools/read_ceiling.c direct: the same reads with O_DIRECT (no page cache)"})
                    res = drop_cache(paths)
                    try:
                        dceil32 = read_ceiling(paths, threads=32, part=8 * MiB, direct=True)
                    except Exception:
                        dceil32 = None
                    emit({"layout": name, "cache": "cold", "read_ceiling_direct_32x8_gbps": round(dceil32 / 1e9, 2)
                          if dceil32 else None, "resident": round(res, 4),
                          "how": "tools/read_ceiling.c direct, 32 threads x 8 MiB requests (more in flight)"})
                for leg, fn, counter in legs:
                    res = drop_cache(paths) if cold else fsutil.resident(paths)
                    if counter is not None:
                        counter.reset()
                    reps = 1 if cold else (3 if leg == "verify_files" else 2)
                    el, bf = timed(fn, reps)
                    rec = {"layout": name, "cache": "cold" if cold else "warm", "path": leg, "resident": round(res, 4),
                           "best_s": round(el, 3), "gbps": round(total / el / 1e9, 2),
                           "exact": bytes(bf) == expect}
                    if counter is not None:
                        rec["gets_per_piece"] = round(counter.gets / reps / P, 3)
                    emit(rec)
                if cold:
                    # the same ceiling after the legs: a storage layer below the page cache (the virtual disk's own
                    # cache) that warms with every pass shows here as a higher figure than before the legs
                    res = drop_cache(paths)
                    ceil2 = read_ceiling(paths)
                    emit({"layout": name, "cache": "cold", "read_ceiling_after_legs_gbps": round(ceil2 / 1e9, 2),
                          "resident": round(res, 4), "how": "tools/read_ceiling.c after the cold legs, after a drop"})
        finally:
            os.chdir(cwd)
        for p in paths:
            os.unlink(p)


if __name__ == "__main__":
    main()
