"""Per-block time of the verify kernel vs piece length / count, with and without a short last piece
(a short last piece hashes in a group of its own, so it must not slow any other group).
usage: python tools/plen_probe.py"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N
for L, P, short in ((256 << 10, 10070, 0), (256 << 10, 10070, 144000), (256 << 10, 10240, 100), (1 << 20, 16384, 0),
                    (1 << 20, 16384, 1000), (64 << 10, 16384, 0), (256 << 10, 65536, 0), (256 << 10, 65536, 5000)):
    for kernel in (1, 2):
        ctx = N.Context(0)
        ctx.set_option(N.TV_OPT_KERNEL, kernel)
        total = L * P - (L - short if short else 0)
        ctx.set_layout(total, L, P)
        ctx.fill_synthetic(1)
        d = bytearray(ctx.hash())
        d[20 * (P - 1)] ^= 1
        ctx.set_digests(bytes(d))
        best = 1e9
        for _ in range(3):
            bf = ctx.verify()
            best = min(best, ctx.last_timing()[0])
        assert bf[-1] & (0x80 >> ((P - 1) % 8)) == 0 and bf[0] & 0x80
        nb = L // 64 + 1
        print(f"{'lane ' if kernel == 1 else 'split'} L={L >> 10:5d} KiB P={P:6d} last={short or L:7d}: kernel {best:7.3f} ms  "
              f"{total / best / 1e6:7.1f} GB/s  {best * 1e-3 * 2.38e9 / nb:6.0f} cyc/block @2.38GHz", flush=True)
        ctx.close()
