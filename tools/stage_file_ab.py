"""tv_stage_file A/B: direct (registered page-cache DMA) vs pinned-ring preads, x window size, page
cache warm, interleaved 4 rounds so box noise hits every variant alike; median GB/s per variant.
usage: python tools/stage_file_ab.py <dir> <GiB> [n_files]"""
import os
import statistics
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

res = {}
for rnd in range(4):
    for mode in (1, 0):
        for chunk in (64 << 20, 256 << 20, 1 << 30):
            ctx.set_option(_native.TV_OPT_FILE_DIRECT, mode)
            ctx.set_option(_native.TV_OPT_FILE_CHUNK, chunk)
            t0 = time.perf_counter()
            for k, path in enumerate(paths):
                assert ctx.stage_file(path, 0, k * per, per)
            el = time.perf_counter() - t0
            res.setdefault((mode, chunk), []).append(total / el / 1e9)
for (mode, chunk), v in sorted(res.items()):
    print(f"direct={mode} chunk={chunk >> 20} MiB: median {statistics.median(v):.2f} GB/s  "
          f"all {[round(x, 1) for x in v]}", flush=True)
ctx.close()
