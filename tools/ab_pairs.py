"""Interleaved A/B (one process): split kernel with 1 vs 2 pairs per workgroup on cfg2."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N
L, P = 1 << 20, 16384
ctx = N.Context(0)
ctx.set_layout(L * P, L, P)
ctx.fill_synthetic(2)
ctx.set_option(N.TV_OPT_KERNEL, 2)
ctx.set_digests(ctx.hash())
res = {1: [], 2: []}
for r in range(6):
    for pairs in (1, 2):
        ctx.set_option(N.TV_OPT_SPLIT_PAIRS, pairs)
        ctx.verify()
        res[pairs].append(ctx.last_timing()[0])
for k, v in res.items():
    v = sorted(v)
    print(f"pairs={k}: median {v[len(v)//2]:.3f} ms min {v[0]:.3f} ms -> {L*P/v[0]/1e6:.0f} GB/s")
