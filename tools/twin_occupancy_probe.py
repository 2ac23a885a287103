"""Per-block time of the twin kernel vs workgroups per CU at a FIXED piece length (1 MiB = 16,384 blocks):
is a twin rounds wave slower when its CU holds one 2-wave workgroup than when it holds two?  And does the
SIMD placement of its helper matter (PROBE_SHAPES=1: TV_OPT_SPLIT_PAIRS 3-5 select probe shapes, tv_kernels.hip)?
And does packing two workgroups on each busy CU (TV_OPT_TWIN_PACK) recover the two-per-CU rate?
usage: python tools/twin_occupancy_probe.py   (one GPU; prints JSON lines)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N  # noqa: E402

L = 1 << 20
for P in [int(x) for x in os.environ.get("PROBE_PS", "4096,6400,8192,12800,16384").split(",")]:
    ctx = N.Context(0)
    ctx.set_layout(L * P, L, P)
    ctx.fill_synthetic(2)
    # pack: bit 0 = TV_OPT_TWIN_PACK, bit 1 = TV_OPT_TWIN_FILL (companion workgroups)
    shapes = [("split1", 2, 1, 0), ("twin1", 4, 1, 0), ("twin1_packed", 4, 1, 1), ("twin1_companions", 4, 1, 2)]
    if os.environ.get("PROBE_SHAPES"):
        shapes += [("twin2", 4, 2, 0), ("twin_r02_h13", 4, 3, 0), ("twin_r0_h2", 4, 4, 0), ("twin_r0_h1", 4, 5, 0)]
    for name, k, pairs, pack in shapes:
        ctx.set_option(N.TV_OPT_KERNEL, k)
        ctx.set_option(N.TV_OPT_SPLIT_PAIRS, pairs)
        ctx.set_option(N.TV_OPT_TWIN_PACK, pack & 1)
        ctx.set_option(N.TV_OPT_TWIN_FILL, pack >> 1)
        ms = []
        for _ in range(6):
            ctx.hash()
            ms.append(ctx.last_timing()[0])
        best = min(ms[1:])
        print(json.dumps({"pieces": P, "kernel": name, "best_ms": round(best, 3),
                          "ns_per_block": round(best * 1e6 / (L // 64 + 1), 2)}), flush=True)
    ctx.close()
