"""Resume-from-disk throughput: write a synthetic multi-file torrent to a directory,
then time verify_files (disk -> pinned -> HBM -> verify).  The files were just written, so the page
cache is warm: this measures the host pipeline + PCIe, not cold NVMe reads.
usage: python tools/resume_bench.py <dir> <GiB> [n_files]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native, make_info, FileInfo, verify_files  # noqa: E402

d, gib = sys.argv[1], float(sys.argv[2])
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 64
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
cwd = os.getcwd()
os.chdir(d)
best = None
for rep in range(3):
    t0 = time.perf_counter()
    bf = verify_files(info, d, threads=16)
    el = time.perf_counter() - t0
    best = el if best is None else min(best, el)
os.chdir(cwd)
ok = all(((bf[i >> 3] >> (7 - (i & 7))) & 1) == (0 if i % 100 == 0 else 1) for i in range(P))
print(f"resume_from_disk: {total / 2**30:.1f} GiB in {nf} files, write {total / wt / 1e9:.2f} GB/s, "
      f"verify_files best {best * 1e3:.0f} ms = {total / best / 1e9:.2f} GB/s (page cache warm), exact={ok}")
