"""Per-call latency of the small-batch paths: verify_piece on one 256 KiB piece through
the cached per-device context (tv_set_layout reuses its allocations), and one tv_verify_list flush of 1, 64
and 4,096 resident 256 KiB pieces (incremental verify, SURVEY 8f row f1: torrent.ts:183-193).

Wall time per call (median of `reps` after warmup) with the library's own HIP-event split: kernel_ms (the
verify kernel) and total_ms (the whole call on the compute stream).  SHA-1 is serial within a piece, so a
256 KiB piece is 4,097 dependent compressions on ONE lane: the kernel time is the floor of every call.
Round 3: each list length with companion workgroups on short lists (TV_OPT_TWIN_FILL 2, the round-2
behaviour) and without (1, auto), twice each, interleaved.
usage: python tools/latency_probe.py [reps]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N  # noqa: E402
from torrent_amd import make_info, verify_piece  # noqa: E402
from torrent_amd.verify import release_contexts  # noqa: E402


def med(xs):
    return round(statistics.median(xs), 3)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import hashlib
    L = 256 << 10
    piece = bytes((i * 131 + 7) & 0xFF for i in range(L))
    info = make_info(L, hashlib.sha1(piece).digest(), "p", length=L)
    out = {}
    # verify_piece: cold (first call creates the context), then warm
    release_contexts()
    t0 = time.perf_counter()
    assert verify_piece(info, 0, piece)
    out["verify_piece_first_call_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    wall = []
    for _ in range(reps):
        t0 = time.perf_counter()
        assert verify_piece(info, 0, piece)
        wall.append((time.perf_counter() - t0) * 1e3)
    out["verify_piece_256k"] = {"wall_ms_median": med(wall), "wall_ms_min": round(min(wall), 3)}
    release_contexts()
    # the same call sequence on a raw context, with the library's timing
    with N.Context(0) as ctx:
        ks, ts, ws = [], [], []
        for _ in range(reps + 2):
            t0 = time.perf_counter()
            ctx.set_layout(L, L, 1, 0, 1)
            ctx.set_digests(hashlib.sha1(piece).digest())
            ctx.stage(0, piece)
            bf = ctx.verify()
            ws.append((time.perf_counter() - t0) * 1e3)
            k, t = ctx.last_timing()
            ks.append(k)
            ts.append(t)
            assert bf == b"\x80"
        out["verify_piece_256k_raw"] = {"wall_ms_median": med(ws[2:]), "kernel_ms_median": med(ks[2:]),
                                        "verify_call_ms_median": med(ts[2:]), "kernel": ctx.last_kernel()[0]}
        # tv_verify_list flushes over a resident shard of 8,192 x 256 KiB pieces
        P = 8192
        ctx.set_layout(P * L, L, P)
        ctx.fill_synthetic(3)
        ctx.set_digests(ctx.hash())
        # TV_OPT_TWIN_FILL 1 (auto: companions only for lists of >= 32 x CUs pieces) against 2 (companions on
        # every list, the round-2 behaviour), interleaved per list length
        for n in (1, 64, 4096, 8192):
            lst = list(range(0, P, P // n))[:n]
            for fill in (1, 2, 1, 2):
                ctx.set_option(N.TV_OPT_TWIN_FILL, fill)
                ws, ks, ts = [], [], []
                for _ in range(reps + 2):
                    t0 = time.perf_counter()
                    ok = ctx.verify_list(lst)
                    ws.append((time.perf_counter() - t0) * 1e3)
                    k, t = ctx.last_timing()
                    ks.append(k)
                    ts.append(t)
                    assert ok == b"\x01" * n
                key = f"verify_list_flush_{n}" + ("" if fill == 1 else "_companions_forced")
                rec = {"wall_ms_median": med(ws[2:]), "kernel_ms_median": med(ks[2:]), "call_ms_median": med(ts[2:]),
                       "workgroups": ctx.counter(N.TV_COUNTER_LAST_WORKGROUPS),
                       "kernel": {1: "lane list", 2: "split list", 4: "twin list"}[ctx.last_kernel()[0]]}
                out.setdefault(key, []).append(rec)
        ctx.set_option(N.TV_OPT_TWIN_FILL, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
