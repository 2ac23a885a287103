"""BASELINE config 3 end to end: 10,000 files of U[0, 512 KiB] bytes (20 zero-length, 5 under 64 B),
256 KiB pieces spanning file boundaries, a short final piece, 1 % corrupted pieces (tests/layouts.py,
expected bitfield committed in tests/golden/layouts.json).

Times (a) verify_payload: the linear payload staged into HBM and verified, (b) verify_files: the
10,000 files written under <dir>, mapped as storage.ts maps them, read by 16 threads into pinned
buffers (every segment is < 32 MiB, so all of them take the pread-run path), staged and verified;
page cache warm.  Every bitfield is checked against the committed expectation.
usage: python tools/cfg3_bench.py <dir>"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.layouts import build_layout, by_name  # noqa: E402
from tests import synth  # noqa: E402
from torrent_amd import verify_files, verify_payload  # noqa: E402
from torrent_amd.verify import _context  # noqa: E402

d = sys.argv[1]
rec = {r["name"]: r for r in json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))}["cfg3"]
t0 = time.perf_counter()
lay = build_layout(by_name("cfg3"), fill=synth.fill)
info = lay["info"]
print(f"cfg3: {len(lay['sizes'])} files, {info.length:,} B, {info.n_pieces} pieces of {info.piece_length} B, "
      f"{len(lay['corrupted'])} corrupted (layout built in {time.perf_counter() - t0:.1f} s)", flush=True)
want = rec["expected_bitfield"]

best = None
for _ in range(5):
    t0 = time.perf_counter()
    bf = verify_payload(info, lay["payload"], avail=lay["avail"])
    el = time.perf_counter() - t0
    assert bytes(bf).hex() == want
    best = el if best is None else min(best, el)
with _context(0) as ctx:
    k_ms, _ = ctx.last_timing()
    kern = ctx.last_kernel()[0]
print(f"verify_payload (host -> HBM stage + verify): best {best * 1e3:.1f} ms = {info.length / best / 1e9:.2f} GB/s; "
      f"verify kernel {k_ms:.2f} ms = {info.length / k_ms / 1e6:.1f} GB/s ({ {1: 'lane', 2: 'split', 3: 'mix', 4: 'twin'}[kern] }); exact", flush=True)

t0 = time.perf_counter()
for path, data in lay["disk_files"]().items():
    p = os.path.join(d, *path)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "wb") as f:
        f.write(data)
print(f"wrote files in {time.perf_counter() - t0:.1f} s", flush=True)
cwd = os.getcwd()
os.chdir(d)
best = None
for _ in range(3):
    t0 = time.perf_counter()
    bf = verify_files(info, d)
    el = time.perf_counter() - t0
    assert bytes(bf).hex() == want
    best = el if best is None else min(best, el)
os.chdir(cwd)
print(f"verify_files (10,000 files, page cache warm): best {best * 1e3:.1f} ms = {info.length / best / 1e9:.2f} GB/s; exact",
      flush=True)
