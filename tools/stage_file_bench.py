"""tv_stage_file throughput: a synthetic torrent written as n files, staged file by file with
tv_stage_file under each TV_OPT_FILE_DIRECT mode, page cache warm and cold (fsync + posix_fadvise
DONTNEED, no root needed), then verified (bitfield exact).
usage: python tools/stage_file_bench.py <dir> <GiB> [n_files]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native  # noqa: E402

d, gib = sys.argv[1], float(sys.argv[2])
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 16
L = 1 << 20
total = int(gib * (1 << 30)) // L * L
P = total // L
per = total // nf
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
ctx.fill_synthetic(7)
pieces = bytearray(ctx.hash())
for i in range(0, P, 100):
    pieces[20 * i] ^= 1
os.makedirs(d, exist_ok=True)
buf = _native.PinnedBuffer(per)
paths = []
for k in range(nf):
    ctx.read(k * per, buf.mv)
    path = os.path.join(d, f"f{k:04d}.bin")
    with open(path, "wb") as fh:
        fh.write(buf.mv)
    paths.append(path)
buf.close()


def evict():
    for path in paths:
        fd = os.open(path, os.O_RDONLY)
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        os.close(fd)


names = {1: "TV_OPT_FILE_DIRECT=1 (warm windows: page-cache DMA; cold: parallel pread)", 0: "TV_OPT_FILE_DIRECT=0 (parallel pread -> pinned ring)"}
for cold in (False, True):
    for mode in (1, 0):
        ctx.set_option(_native.TV_OPT_FILE_DIRECT, mode)
        best = None
        for rep in range(2):
            ctx.set_layout(total, L, P)
            ctx.set_digests(bytes(pieces))
            if cold:
                evict()
            t0 = time.perf_counter()
            for k, path in enumerate(paths):
                assert ctx.stage_file(path, 0, k * per, per)
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        bf = ctx.verify()
        ok = all(((bf[i >> 3] >> (7 - (i & 7))) & 1) == (0 if i % 100 == 0 else 1) for i in range(P))
        print(f"stage_file {total / 2**30:.0f} GiB / {nf} files, {'COLD' if cold else 'warm'}, {names[mode]}: "
              f"{best * 1e3:.0f} ms = {total / best / 1e9:.2f} GB/s, exact={ok}", flush=True)
ctx.close()
