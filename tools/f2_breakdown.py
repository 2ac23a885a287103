"""Where verify_files' time goes on BASELINE cfg3 (10,000 files, page cache warm): host preparation (the
storage.ts walk, paths), tv_stage_files (reads by the library's threads into pinned slots + DMA), tv_verify
(the kernel), for TV_OPT_FILE_THREADS = 4, 8, 16.  Every bitfield is checked against the committed one.
Then the two halves of tv_stage_files alone: the DMA (tv_stage of the same linear bytes from a page-locked
buffer: 2D copies at pitch stride) and the reads (16 Python threads doing open/preadv/close of the 10,000
files into one buffer, no DMA).
usage: python tools/f2_breakdown.py <dir>"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.layouts import build_layout, by_name  # noqa: E402
from tests import synth  # noqa: E402
from torrent_amd import _native, verify_files  # noqa: E402

d = sys.argv[1]
rec = {r["name"]: r for r in json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))}["cfg3"]
lay = build_layout(by_name("cfg3"), fill=synth.fill)
info = lay["info"]
for path, data in lay["disk_files"]().items():
    p = os.path.join(d, *path)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "wb") as f:
        f.write(data)
os.chdir(d)

acc = {"stage_files": 0.0, "verify": 0.0}
orig_stage, orig_verify = _native.Context.stage_files, _native.Context.verify


def stage_files(self, *a, **k):
    t = time.perf_counter()
    r = orig_stage(self, *a, **k)
    acc["stage_files"] += time.perf_counter() - t
    return r


def verify(self, *a, **k):
    t = time.perf_counter()
    r = orig_verify(self, *a, **k)
    acc["verify"] += time.perf_counter() - t
    return r


_native.Context.stage_files, _native.Context.verify = stage_files, verify
for threads in (4, 8, 16):
    best = None
    for _ in range(4):
        acc["stage_files"] = acc["verify"] = 0.0
        t0 = time.perf_counter()
        bf = verify_files(info, d, threads=threads)
        el = time.perf_counter() - t0
        assert bytes(bf).hex() == rec["expected_bitfield"]
        row = {"total_ms": el * 1e3, "stage_files_ms": acc["stage_files"] * 1e3, "verify_ms": acc["verify"] * 1e3}
        row["host_prep_ms"] = row["total_ms"] - row["stage_files_ms"] - row["verify_ms"]
        if best is None or el * 1e3 < best["total_ms"]:
            best = row
    best = {k: round(v, 2) for k, v in best.items()}
    best["threads"] = threads
    best["stage_GBps"] = round(info.length / best["stage_files_ms"] / 1e6, 2)
    best["GBps"] = round(info.length / best["total_ms"] / 1e6, 2)
    print(json.dumps(best), flush=True)

# the DMA alone: the linear payload from page-locked memory
L, P, total = info.piece_length, info.n_pieces, info.length
pb = _native.PinnedBuffer(total)
pb.mv[:] = lay["payload"][:total]
with _native.Context(0) as ctx:
    ctx.set_layout(total, L, P)
    best = None
    for _ in range(5):
        t = time.perf_counter()
        ctx.stage(0, pb.mv)
        el = time.perf_counter() - t
        best = el if best is None else min(best, el)
print(json.dumps({"dma_from_pinned_ms": round(best * 1e3, 2), "GBps": round(total / best / 1e9, 2)}), flush=True)

# the reads alone: open / preadv / close of every file into one buffer on 16 threads
from concurrent.futures import ThreadPoolExecutor  # noqa: E402
from torrent_amd.storage import Storage, fs_storage  # noqa: E402
st = Storage(fs_storage, info, d)
k, foff, nbytes, start = st.segment_arrays(0, total)
paths = st.file_paths()
buf = bytearray(total)
mv = memoryview(buf)
jobs = [(paths[int(a)], int(b), int(c), int(e)) for a, b, c, e in zip(k, foff, nbytes, start)]


def read(job):
    path, fo, n, lin = job
    fd = os.open(path, os.O_RDONLY)
    try:
        got = os.preadv(fd, [mv[lin:lin + n]], fo)
    finally:
        os.close(fd)
    return got == n


for threads in (4, 16):
    best = None
    with ThreadPoolExecutor(threads) as ex:
        for _ in range(4):
            t = time.perf_counter()
            assert all(ex.map(read, jobs, chunksize=64))
            el = time.perf_counter() - t
            best = el if best is None else min(best, el)
    print(json.dumps({"python_reads_threads": threads, "ms": round(best * 1e3, 2), "GBps": round(total / best / 1e9, 2)}),
          flush=True)
