"""Does the destination memory set the rate of cold O_DIRECT reads?  A file is written (tests/synth.py bytes), dropped
from the page cache (residency checked), and read whole with O_DIRECT by `threads` threads in 4 MiB requests into a
256 MiB destination of each kind, interleaved over two rounds:
  pinned        tv_host_alloc (hipHostMalloc: the library's staging ring memory)
  anon_thp      anonymous mmap with MADV_HUGEPAGE (transparent huge pages), touched first
  anon_4k       anonymous mmap with MADV_NOHUGEPAGE, touched first
  thp_register  anon_thp, then tv_host_register (page-locked for the GPU's DMA, as a THP ring would be)
One JSON line per (round, destination, threads).

    python tools/odirect_dest_probe.py DIR [gib] [threads,...]
"""
import ctypes
import json
import mmap
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fsutil  # noqa: E402
from tests import synth  # noqa: E402
from torrent_amd import _native  # noqa: E402

MiB = 1 << 20
PART = 4 * MiB
DEST = 256 * MiB
_libc = ctypes.CDLL(None, use_errno=True)
_libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE, MADV_NOHUGEPAGE = 14, 15


def anon(huge):
    m = mmap.mmap(-1, DEST, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
    _libc.madvise(addr, DEST, MADV_HUGEPAGE if huge else MADV_NOHUGEPAGE)
    for o in range(0, DEST, 4096):
        m[o] = 1
    return m, addr


def read_all(path, size, addr, threads):
    fd = os.open(path, os.O_RDONLY | os.O_DIRECT)
    nparts = size // PART
    nxt = [0]
    lock = threading.Lock()
    err = []

    def worker():
        buf_type = ctypes.c_char * PART
        while True:
            with lock:
                q = nxt[0]
                nxt[0] += 1
            if q >= nparts:
                return
            dst = buf_type.from_address(addr + (q % (DEST // PART)) * PART)
            got = os.preadv(fd, [memoryview(dst).cast("B")], q * PART)
            if got != PART:
                err.append(got)
                return

    t = time.perf_counter()
    ths = [threading.Thread(target=worker) for _ in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t
    os.close(fd)
    return (size / el / 1e9) if not err else None


def main():
    d = sys.argv[1]
    gib = float(sys.argv[2]) if len(sys.argv) > 2 else 8
    thread_list = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "4,8").split(",")]
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "odirect_probe.bin")
    size = int(gib * (1 << 30)) // PART * PART
    with open(path, "wb") as f:
        for o in range(0, size, 256 * MiB):
            f.write(synth.fill(5, o, min(256 * MiB, size - o)))
    pinned = _native.PinnedBuffer(DEST)
    thp, thp_addr = anon(True)
    a4k, a4k_addr = anon(False)
    reg, reg_addr = anon(True)
    if _native.lib().tv_host_register(reg_addr, DEST) != 0:
        reg_addr = None
    dests = [("pinned", pinned.ptr), ("anon_thp", thp_addr), ("anon_4k", a4k_addr)]
    if reg_addr:
        dests.append(("thp_register", reg_addr))
    for rnd in range(2):
        for threads in thread_list:
            for name, addr in dests:
                res = fsutil.drop_cache([path])
                rec = {"round": rnd, "dest": name, "threads": threads, "resident": round(res, 4)}
                if res <= 0.01:
                    g = read_all(path, size, addr, threads)
                    rec["gbps"] = round(g, 2) if g else None
                print(json.dumps(rec), flush=True)
    os.unlink(path)


if __name__ == "__main__":
    main()
