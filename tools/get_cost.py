"""What one fsStorage.get costs on cfg3's 10,000 small files (the reference-shaped Storage path's bound):
every piece's Storage(fs).get on 1 and 16 threads, page cache warm, for fsStorage variants that return the same
bytes:
  ref       torrent_amd.storage.FsStorage: open(O_RDWR | O_CREAT) + pread + close, as storage.ts:149-172
  nocreat   open(O_RDWR) first, O_CREAT only when the file is missing (the same file state afterwards)
  rdonly    open(O_RDONLY) + pread + close (not the reference's semantics: the floor of an open per get)
  openonly  the open and close alone, no read
Prints one JSON line per (variant, threads): gets, wall seconds, microseconds per get (wall / gets, i.e. the
aggregate rate), GB/s of piece bytes.

    python tools/get_cost.py DIR [cfg3|single16|files64] [sweep]"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from storage_paths_bench import write_layout  # noqa: E402
from torrent_amd import Storage  # noqa: E402
from torrent_amd.piece import piece_length  # noqa: E402
from torrent_amd.storage import FsStorage  # noqa: E402


class NoCreat(FsStorage):
    def get(self, path, offset, length):
        p = os.path.join(*path)
        try:
            try:
                fd = os.open(p, os.O_RDWR)
            except FileNotFoundError:
                fd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
        except OSError:
            return None
        try:
            data = os.pread(fd, length, offset) if length else b""
            return data if len(data) == length else None
        except OSError:
            return None
        finally:
            os.close(fd)


class RdOnly(FsStorage):
    def get(self, path, offset, length):
        try:
            fd = os.open(os.path.join(*path), os.O_RDONLY)
        except OSError:
            return None
        try:
            data = os.pread(fd, length, offset) if length else b""
            return data if len(data) == length else None
        finally:
            os.close(fd)


class OpenOnly(FsStorage):
    def get(self, path, offset, length):
        try:
            fd = os.open(os.path.join(*path), os.O_RDWR | os.O_CREAT, 0o644)
        except OSError:
            return None
        os.close(fd)
        return bytes(length) if length <= 4096 else memoryview(_ZERO)[:length]


_ZERO = bytes(1 << 20)


class Counting:
    def __init__(self, inner):
        self.inner, self.gets = inner, 0

    def get(self, path, offset, length):
        self.gets += 1          # (racy under threads; the count of the 1-thread run is used)
        return self.inner.get(path, offset, length)


def main():
    d = sys.argv[1]
    layout = sys.argv[2] if len(sys.argv) > 2 else "cfg3"
    sweep = len(sys.argv) > 3 and sys.argv[3] == "sweep"   # the reference method over 1 .. 16 threads only
    root = os.path.join(d, layout)
    info, _, paths = write_layout(layout, root)
    P, L = info.n_pieces, info.piece_length
    os.chdir(root)
    gets = None
    variants = (("ref", FsStorage()),) if sweep else (("ref", FsStorage()), ("nocreat", NoCreat()), ("rdonly", RdOnly()),
                                                       ("openonly", OpenOnly()))
    for name, method in variants:
        for threads in ((1, 2, 4, 8, 16) if sweep else (1, 16)):
            cm = Counting(method)
            st = Storage(cm, info, root)
            best = None
            for _ in range(2):
                t0 = time.perf_counter()
                with ThreadPoolExecutor(threads) as ex:
                    n_ok = sum(ex.map(lambda i: st.get(i * L, piece_length(i, info)) is not None, range(P)))
                el = time.perf_counter() - t0
                best = el if best is None else min(best, el)
            if gets is None:
                gets = cm.gets // 2
            print(json.dumps({"layout": layout, "variant": name, "threads": threads, "gets": gets, "pieces_ok": n_ok,
                              "best_s": round(best, 4), "us_per_get": round(best / gets * 1e6, 2),
                              "gbps": round(info.length / best / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
