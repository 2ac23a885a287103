"""Where does verify_files spend its time on a many-small-files torrent (BASELINE cfg3: 10,000 files)?
Times each step of one shard: set_layout, set_digests, the storage.ts segment mapping, ONE
tv_stage_files call (reader pool), verify.  Page cache warm.
usage: python tools/stage_files_probe.py <dir>"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.layouts import build_layout, by_name  # noqa: E402
from tests import synth  # noqa: E402
from torrent_amd import _native  # noqa: E402
from torrent_amd.storage import Storage, fs_storage  # noqa: E402

d = sys.argv[1]
lay = build_layout(by_name("cfg3"), fill=synth.fill)
info = lay["info"]
for path, data in lay["disk_files"]().items():
    p = os.path.join(d, *path)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "wb") as f:
        f.write(data)
os.chdir(d)
L, P = info.piece_length, info.n_pieces
ctx = _native.Context(0)
for rep in range(3):
    t = [time.perf_counter()]
    ctx.set_layout(info.length, L, P)
    t.append(time.perf_counter())
    ctx.set_digests(info.pieces_raw)
    t.append(time.perf_counter())
    segs = [sg for sg in Storage(fs_storage, info, d).segments(0, info.length) if sg[2] > 0]
    args = ([os.path.join(*p) for p, _, _, _ in segs], [fo for _, fo, _, _ in segs], [s0 for _, _, _, s0 in segs],
            [n for _, _, n, _ in segs])
    t.append(time.perf_counter())
    for threads in ((1, 2, 4, 8, 16) if rep == 2 else (16,)):
        ctx.set_option(_native.TV_OPT_FILE_THREADS, threads)
        a = time.perf_counter()
        st = ctx.stage_files(*args)
        if rep == 2:
            print(f"  threads={threads}: stage_files {info.length / (time.perf_counter() - a) / 1e9:.2f} GB/s", flush=True)
    t.append(time.perf_counter())
    bf = ctx.verify()
    t.append(time.perf_counter())
    names = ["set_layout", "set_digests", "segments", "stage_files", "verify"]
    print(f"rep {rep}: " + ", ".join(f"{n} {(b - a) * 1e3:.1f} ms" for n, a, b in zip(names, t, t[1:])) +
          f"; stage_files {info.length / (t[4] - t[3]) / 1e9:.2f} GB/s over {len(segs)} segments; io errors "
          f"{sum(1 for x in st if x)}", flush=True)
ctx.close()
