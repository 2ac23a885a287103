"""Scratch throughput probe: fill a synthetic shard on device, hash it, verify it, per kernel."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N

def run(total, L, kernels=(1, 2), reps=3, pad=None):
    P = -(-total // L)
    ctx = N.Context(0)
    if pad: ctx.set_option(N.TV_OPT_STRIDE_PAD, pad)
    ctx.set_layout(total, L, P)
    ctx.fill_synthetic(2)
    for k in kernels:
        ctx.set_option(N.TV_OPT_KERNEL, k)
        d = ctx.hash()
        ctx.set_digests(d)
        best = 1e9
        for _ in range(reps):
            bf = ctx.verify()
            km, tm = ctx.last_timing()
            best = min(best, km)
        ok = all(b == 0xFF for b in bf[:-1])
        print(f"total={total/2**30:.2f}GiB L={L>>10}KiB P={P} kernel={k} pad={pad} kernel_ms={best:.3f} "
              f"GB/s={total/best/1e6:.1f} allones={ok}", flush=True)
    ctx.close()

if __name__ == "__main__":
    import sys as _s
    which = _s.argv[1] if len(_s.argv) > 1 else "all"
    if which in ("all", "cfg2"):
        run(16 << 30, 1 << 20)           # cfg2: 16384 pieces
    if which in ("all", "mid"):
        run(25 << 30, 1 << 20)           # 25600 pieces (cfg4 per GPU at N=2, 1 MiB pieces)
        run(16 << 30, 512 << 10)         # 32768 pieces
        run(20 << 30, 512 << 10)         # 40960 pieces
        run(16 << 30, 256 << 10)         # 65536 pieces
    if which in ("all", "big"):
        run(16 << 30, 64 << 10, (1,))    # 262144 pieces (lane)
        run(50 << 30, 4 << 20)           # 12800 pieces x 4 MiB (cfg4 per GPU at N=4)
