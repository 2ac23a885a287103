"""Where the split (and twin, --kernel 4) kernel's waves spend their cycles, from in-kernel clock stamps (VERDICT r03
item 5).

A diagnostic library (tools/build_variants.py stamps:STAMP=1,D_TV_STAMPS=1 -> build/variants/libtv_stamps.so)
brackets every in-loop workgroup barrier of the split kernel's rounds and helper waves with `s_memtime` reads and
accumulates the cycles spent there in an SGPR; each wave also times its whole asm loop.  STAMP=2 builds also
bracket the helper's two waits per block (its prefetched global words: vmcnt; its LDS writes before the barrier:
lgkmcnt).  Per workgroup and wave the library leaves {loop cycles, barrier cycles, loop blocks, 1, vmcnt cycles,
lgkmcnt cycles} after the clock probe's words (tv_debug_stamps).

    TORRENT_VERIFY_LIB=build/variants/libtv_stamps.so python tools/split_stamps.py [--pieces 51200]
        [--piece-mib 4] [--shards 2] [--reps 3]

Runs the split kernel (TV_OPT_KERNEL 2) on one rank's shard (default: cfg4 at N = 2, 25,600 x 4 MiB), checks every
bit, and prints one JSON line: kernel ms, the clock, and per wave role the loop cycles per block, the barrier cycles
per block (mean and the 10/50/90th percentiles over workgroups) and the rest (the wave's own instruction stream).
Each stamp costs the waves two s_memtime reads and one wait per block; the kernel time beside the shipped
library's (run the same command without TORRENT_VERIFY_LIB, which has no stamps and reports `stamps: null`) is
that perturbation."""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from torrent_amd import _native as N  # noqa: E402
from torrent_amd.verify import shard_ranges  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=51200)
    ap.add_argument("--piece-mib", type=int, default=4)
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kernel", type=int, default=2, help="2 split, 4 twin (the 2-wave shape: wave 0 rounds, 1 helper)")
    a = ap.parse_args()
    L = a.piece_mib << 20
    P = a.pieces
    first, count = shard_ranges(P, a.shards)[0]
    stamped = hasattr(N.lib(), "tv_debug_stamps")
    out = {"kernel": a.kernel, "pieces_per_gpu": count, "piece_length": L, "lib": os.path.relpath(N.LIB_PATH, ROOT), "stamped": stamped}
    with N.Context(0) as ctx:
        ctx.set_option(N.TV_OPT_KERNEL, a.kernel)
        ctx.set_option(N.TV_OPT_CLOCK_PROBE, 1)
        ctx.set_layout(L * P, L, P, first, count)
        ctx.fill_synthetic(4)
        dig = bytearray(ctx.hash())
        bad = set(range(3, count, 100))
        for j in bad:
            dig[20 * j + 5] ^= 0x08
        pieces = bytearray(20 * P)
        pieces[20 * first:20 * (first + count)] = dig
        ctx.set_digests(bytes(pieces))
        ms, clocks, reps = [], [], []
        wgs = 0
        for k in range(a.warmup + a.reps):
            bf = ctx.verify()
            exact = all(((bf[j >> 3] >> (7 - (j & 7))) & 1) == (0 if j in bad else 1) for j in range(count))
            assert exact, "bitfield differs from the expected one"
            if k < a.warmup:
                continue
            ms.append(ctx.last_timing()[0])
            clocks.append(ctx.counter(N.TV_COUNTER_LAST_CLOCK_KHZ) / 1e6)
            wgs = ctx.counter(N.TV_COUNTER_LAST_WORKGROUPS)
            if stamped:
                words = 4 + 32 * wgs
                buf = (ctypes.c_uint64 * words)()
                fn = N.lib().tv_debug_stamps
                fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
                ctx._check(fn(ctx._h, buf, ctypes.sizeof(buf)))
                reps.append([tuple(buf[4 + 8 * i:12 + 8 * i]) for i in range(4 * wgs)])
        assert ctx.last_kernel()[0] == a.kernel, "the requested kernel did not run"
    out.update({"workgroups": wgs, "kernel_ms": [round(x, 3) for x in ms], "kernel_ms_median": round(statistics.median(ms), 3),
                "gbps": round(L * count / (statistics.median(ms) / 1e3) / 1e9, 1),
                "clock_ghz": [round(c, 3) for c in clocks]})
    if stamped:
        roles = {}
        for role, name in ((0, "rounds"), (1, "helper")):
            loop, bar, vm, lg = [], [], [], []
            for rep in reps:
                for g in range(wgs):
                    lc, bc, nb, valid, vc, gc = rep[4 * g + role][:6]
                    if valid and nb:
                        loop.append(lc / nb)
                        bar.append(bc / nb)
                        vm.append(vc / nb)
                        lg.append(gc / nb)
            roles[name] = {"waves": len(loop) // len(reps),
                           "loop_cycles_per_block": round(statistics.mean(loop), 1),
                           "barrier_cycles_per_block": round(statistics.mean(bar), 1),
                           "barrier_p10_p50_p90": [round(pct(bar, q), 1) for q in (0.1, 0.5, 0.9)],
                           "rest_cycles_per_block": round(statistics.mean(loop) - statistics.mean(bar), 1)}
            if role == 1 and any(vm):
                roles[name].update({"vmcnt_wait_cycles_per_block": round(statistics.mean(vm), 1),
                                    "lgkmcnt_wait_cycles_per_block": round(statistics.mean(lg), 1),
                                    "rest_cycles_per_block": round(statistics.mean(loop) - statistics.mean(bar)
                                                                   - statistics.mean(vm) - statistics.mean(lg), 1)})
        out["stamps"] = roles
    else:
        out["stamps"] = None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
