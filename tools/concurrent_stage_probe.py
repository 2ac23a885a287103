"""Can the two warm file-staging mechanisms run side by side? Two contexts on one GPU stage half of a
16 GiB / 64-file torrent each, concurrently: one through the tv_stage_file path (page-cache pages
registered and DMA'd), one through the reader pool (preads into pinned slots).  Aggregate vs alone.
usage: python tools/concurrent_stage_probe.py <dir>"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native  # noqa: E402

d = sys.argv[1]
L, nf = 1 << 20, 64
per = 256 << 20
total = per * nf
P = total // L
os.makedirs(d, exist_ok=True)
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
ctx.fill_synthetic(3)
buf = _native.PinnedBuffer(per)
paths = []
for k in range(nf):
    ctx.read(k * per, buf.mv)
    p = os.path.join(d, f"f{k:03d}.bin")
    with open(p, "wb") as f:
        f.write(buf.mv)
    paths.append(p)
buf.close()
ctx.close()
half = nf // 2


def make(first_file, direct_min):
    c = _native.Context(0)
    c.set_layout(total, L, P)
    c.set_option(_native.TV_OPT_FILE_DIRECT_MIN, direct_min)
    ks = range(first_file, first_file + half)
    args = ([paths[k] for k in ks], [0] * half, [k * per for k in ks], [per] * half)
    return c, args


a, aa = make(0, 0)           # direct
b, ba = make(half, 1 << 62)  # reader pool
for label, jobs in (("direct alone", [(a, aa)]), ("pool alone", [(b, ba)]), ("both at once", [(a, aa), (b, ba)])):
    best = 1e9
    for _ in range(3):
        ths = [threading.Thread(target=c.stage_files, args=args) for c, args in jobs]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        best = min(best, time.perf_counter() - t0)
    print(f"{label:14s}: {len(jobs) * half * per / best / 1e9:6.2f} GB/s", flush=True)
a.close()
b.close()
