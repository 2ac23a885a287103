"""Resume-from-disk throughput: write a synthetic multi-file torrent to a directory,
then time verify_files (disk -> HBM -> verify; one tv_stage_files call) with its two staging paths:
direct (the tv_stage_file path: page-cache pages DMA'd to HBM) and the reader pool (library threads
pread into pinned slots, then DMA).  Each
is timed with the page cache warm (the files were just written) and cold (posix_fadvise DONTNEED
after fsync, so the reads go to the box's disk).
With --lanes-ab: only the warm direct case, one staging lane against two (TV_OPT_FILE_CONCURRENT on
the cached context), interleaved over 6 rounds.
usage: python tools/resume_bench.py <dir> <GiB> [n_files] [--warm-only|--pread-first|--lanes-ab]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import statistics  # noqa: E402

from torrent_amd import _native, make_info, FileInfo, verify_files  # noqa: E402
from torrent_amd.verify import _context  # noqa: E402

d, gib = sys.argv[1], float(sys.argv[2])
nf = int(sys.argv[3]) if len(sys.argv) > 3 and not sys.argv[3].startswith("-") else 64
L = 1 << 20
total = int(gib * (1 << 30)) // L * L
P = total // L
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
ctx.fill_synthetic(5)
pieces = bytearray(ctx.hash())
for i in range(0, P, 100):
    pieces[20 * i] ^= 1
per = total // nf
sizes = [per] * (nf - 1) + [total - per * (nf - 1)]
files = [FileInfo(s, [f"f{k:04d}.bin"]) for k, s in enumerate(sizes)]
info = make_info(L, bytes(pieces), "r", files=files)
os.makedirs(d, exist_ok=True)
buf = _native.PinnedBuffer(max(sizes))
off = 0
t0 = time.perf_counter()
for f in files:
    mv = buf.mv[:f.length]
    ctx.read(off, mv)
    with open(os.path.join(d, *f.path), "wb") as fh:
        fh.write(mv)
    off += f.length
buf.close()
ctx.close()
wt = time.perf_counter() - t0


def evict():
    """Drop the files' clean pages from the page cache (posix_fadvise DONTNEED: no root needed)."""
    for f in files:
        fd = os.open(os.path.join(d, *f.path), os.O_RDONLY)
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        os.close(fd)


def exact(bf):
    return all(((bf[i >> 3] >> (7 - (i & 7))) & 1) == (0 if i % 100 == 0 else 1) for i in range(P))


cwd = os.getcwd()
os.chdir(d)
if "--lanes-ab" in sys.argv:
    res = {1: [], 2: []}
    for rnd in range(6):
        for lanes in (2, 1):
            with _context(0) as c:
                c.set_option(_native.TV_OPT_FILE_CONCURRENT, lanes - 1)
            t0 = time.perf_counter()
            bf = verify_files(info, d, threads=16)
            el = time.perf_counter() - t0
            assert exact(bf)
            res[lanes].append(total / el / 1e9)
    for lanes, v in res.items():
        print(f"resume_from_disk: {total / 2**30:.1f} GiB in {nf} files, page cache warm, direct, {lanes} staging "
              f"lane(s): median {statistics.median(v):.2f} GB/s, best {max(v):.2f}  all {[round(x, 1) for x in v]}",
              flush=True)
    sys.exit(0)
modes = [("direct (tv_stage_file path: page-cache DMA)", None), ("reader pool (preads -> pinned slots -> DMA)", 1 << 62)]
if "--pread-first" in sys.argv:
    modes = modes[::-1] + modes[1:]
for cold in ((False,) if "--warm-only" in sys.argv else (False, True)):
    for name, dmin in modes:
        best, ok = None, True
        for rep in range(2 if cold else 3):
            if cold:
                evict()
            t0 = time.perf_counter()
            bf = verify_files(info, d, threads=16, direct_min=dmin)
            el = time.perf_counter() - t0
            ok = ok and exact(bf)
            best = el if best is None else min(best, el)
        print(f"resume_from_disk: {total / 2**30:.1f} GiB in {nf} files, write {total / wt / 1e9:.2f} GB/s, "
              f"{'COLD (fadvise DONTNEED)' if cold else 'page cache warm'}, {name}: best {best * 1e3:.0f} ms = "
              f"{total / best / 1e9:.2f} GB/s, exact={ok}", flush=True)
os.chdir(cwd)
