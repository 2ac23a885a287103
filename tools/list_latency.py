"""Incremental-verify latency: one tv_verify_list call over n just-completed pieces
of a resident 256 KiB-piece shard, lane list kernel vs split kernel in list mode.  Reports the kernel
time (HIP events) and the whole call, median of 7.
usage: python tools/list_latency.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native  # noqa: E402

L, P = 256 << 10, 16384
ctx = _native.Context(0)
ctx.set_layout(L * P, L, P)
ctx.fill_synthetic(3)
ctx.set_digests(ctx.hash())
for n in (1, 16, 64, 256, 1024, 4096, 16384):
    lst = list(range(0, P, max(1, P // n)))[:n]
    row = []
    for kernel in (1, 2):
        ctx.set_option(_native.TV_OPT_KERNEL, kernel)
        ks, ts = [], []
        for _ in range(7):
            ok = ctx.verify_list(lst)
            k, t = ctx.last_timing()
            ks.append(k)
            ts.append(t)
        assert ok == b"\x01" * n
        row.append(f"{'lane' if kernel == 1 else 'split'} kernel {statistics.median(ks):7.3f} ms "
                   f"call {statistics.median(ts):7.3f} ms")
    print(f"n={n:6d} x 256 KiB: " + " | ".join(row), flush=True)
ctx.close()
