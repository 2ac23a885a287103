"""H2D staging rate from pinned host memory vs source/destination alignment (tv_stage from a
tv_host_alloc buffer: direct DMA, one 2D copy per run of whole pieces).
usage: python tools/dma_align_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native  # noqa: E402

L, P = 256 << 10, 4096
ctx = _native.Context(0)
ctx.set_layout(L * P, L, P)
pb = _native.PinnedBuffer(L * P + 8192)
n = 64 << 20
for src_off, lin_off in ((0, 0), (1, 0), (100, 0), (4096, 0), (0, 100), (100, 100), (4196, 100), (1000, 77777)):
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        for r in range(4):
            ctx.stage(lin_off + r * n, pb.mv[src_off + r * n % 8192:src_off + r * n % 8192 + n])
        best = min(best, time.perf_counter() - t0)
    print(f"src offset {src_off:5d} (mod 256 = {src_off % 256:3d}), linear offset {lin_off:6d} (mod 256 = {lin_off % 256:3d}): "
          f"{4 * n / best / 1e9:6.2f} GB/s", flush=True)
pb.close()
ctx.close()
