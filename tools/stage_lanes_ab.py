"""tv_stage_files with one staging lane against two (TV_OPT_FILE_CONCURRENT), page cache warm: a
16 GiB torrent in 64 files of 256 MiB (every segment long: the tv_stage_file path), and the same
with half the files cut into 4 MiB pieces of their own (long segments beside the reader pool).
Interleaved rounds so box noise hits every variant alike; median GB/s per variant; every staged
payload is checked by hashing it on the GPU against the digests of the first round.
usage: python tools/stage_lanes_ab.py <dir>"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native  # noqa: E402

d = sys.argv[1]
L, nf, per = 1 << 20, 64, 256 << 20
total = per * nf
P = total // L
os.makedirs(d, exist_ok=True)
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
ctx.fill_synthetic(3)
want = ctx.hash()
buf = _native.PinnedBuffer(per)
big, small = [], []
for k in range(nf):
    ctx.read(k * per, buf.mv)
    if k % 2 == 0:
        p = os.path.join(d, f"f{k:03d}.bin")
        with open(p, "wb") as f:
            f.write(buf.mv)
        big.append((p, 0, k * per, per))
    else:
        for q in range(0, per, 4 << 20):
            p = os.path.join(d, f"f{k:03d}_{q >> 22:03d}.bin")
            with open(p, "wb") as f:
                f.write(buf.mv[q:q + (4 << 20)])
            small.append((p, 0, k * per + q, 4 << 20))
buf.close()
# layout "long": the 32 big files plus the 32 others as whole 256 MiB files (written once more)
longs = list(big)
for k in range(1, nf, 2):
    p = os.path.join(d, f"g{k:03d}.bin")
    with open(p, "wb") as f:
        for q in range(0, per, 4 << 20):
            with open(os.path.join(d, f"f{k:03d}_{q >> 22:03d}.bin"), "rb") as g:
                f.write(g.read())
    longs.append((p, 0, k * per, per))
layouts = {"64 x 256 MiB": longs, "32 x 256 MiB + 2048 x 4 MiB": big + small}

res = {}
for rnd in range(4):
    for name, segs in layouts.items():
        for conc in (1, 0):
            ctx.set_option(_native.TV_OPT_FILE_CONCURRENT, conc)
            ctx.fill_synthetic(1)
            args = [list(x) for x in zip(*segs)]
            t0 = time.perf_counter()
            st = ctx.stage_files(*args)
            el = time.perf_counter() - t0
            assert st == [0] * len(segs)
            assert ctx.hash() == want, (name, conc)
            res.setdefault((name, conc), []).append(total / el / 1e9)
for (name, conc), v in res.items():
    print(f"{name:28s} lanes={2 if conc else 1}: median {statistics.median(v):.2f} GB/s  all {[round(x, 1) for x in v]}",
          flush=True)
ctx.close()
