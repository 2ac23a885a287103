"""What a windowed layout costs: verify_payload over a payload in page-locked host memory with the whole shard
resident (one window) and under smaller device budgets (TV_OPT_RESIDENT_BUDGET: windows of pieces staged while the
previous window hashes), beside the streamed path (verify_stream over the same memory).  Every bitfield is checked
against hashlib's digests of the payload (1 % of them corrupted; tests/synth.py generates it).

    python tools/window_bench.py [--gib 16] [--piece-mib 1] [--budgets 0,8,2,0.5] [--reps 3] [--variants 4:0,2:1]
                                 [--files DIR [--cold [--cold-variants 512:0,2048:16]]]

--variants: window buffers : hash streams (TV_OPT_WIN_BUFS / TV_OPT_WIN_STREAMS; 0 = the library's default) tried
on every windowed budget (round 6: windows hashed side by side on hash streams of their own).

Prints one JSON line per leg: path, budget (GiB; 0 = automatic), windows and window pieces (the library's
counters), best and median wall seconds of the call, GB/s (payload bytes / best wall, H2D included)."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import synth  # noqa: E402  (the generator and hashlib digests: nothing under oracle/ runs here)
from torrent_amd import _native as N  # noqa: E402
from torrent_amd.metainfo import make_info  # noqa: E402
from torrent_amd.verify import _context, context_counters, verify_payload, verify_stream  # noqa: E402

GiB, MiB = 1 << 30, 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16)
    ap.add_argument("--piece-mib", type=float, default=1)
    ap.add_argument("--budgets", default="0,8,2,0.5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="0:0")
    ap.add_argument("--files", default=None,
                    help="also verify_files on a warm single16 layout (one 16 GiB file, 1 MiB pieces) written to this dir")
    ap.add_argument("--cold", action="store_true",
                    help="with --files: also cold legs (the file evicted from the page cache before each rep)")
    ap.add_argument("--cold-variants", default="0:0",
                    help="cold streamed legs: pieces per window : reader threads [: KiB per request] "
                         "(TV_OPT_STREAM_COLD_WINDOW / _READERS / _REQ; 0 = the library's default)")
    a = ap.parse_args()
    L = int(a.piece_mib * MiB)
    total = int(a.gib * GiB) // L * L
    P = total // L
    seed = 7
    buf = N.PinnedBuffer(total)
    chunk = 256 * MiB
    for o in range(0, total, chunk):
        n = min(chunk, total - o)
        ctypes.memmove(buf.ptr + o, bytes(synth.fill(seed, o, n)), n)
    digests = bytearray(synth.piece_digests(seed, total, L, P, threads=16))
    for i in range(5, P, 100):
        digests[20 * i + 3] ^= 0x08
    expect = bytearray(b"\xff" * ((P + 7) // 8))
    for i in range(5, P, 100):
        expect[i >> 3] &= ~(0x80 >> (i & 7)) & 0xFF
    if P % 8:
        expect[-1] &= (0xFF << (8 - P % 8)) & 0xFF
    info = make_info(L, bytes(digests), "w", length=total)

    def leg(name, fn, budget_gib, variant=None, pre=None):
        walls, ok, res = [], True, []
        for _ in range(a.reps):
            if pre:
                res.append(pre())
            t0 = time.perf_counter()
            bf = fn()
            walls.append(time.perf_counter() - t0)
            ok &= bytes(bf) == bytes(expect)
        cnt = next(iter(context_counters().values()), {})
        with _context(0) as ctx:
            wb, ws = ctx.counter(N.TV_COUNTER_WINDOW_BUFS), ctx.counter(N.TV_COUNTER_WINDOW_STREAMS)
        print(json.dumps({"path": name, "bytes": total, "piece_length": L, "pieces": P, "budget_gib": budget_gib,
                          "variant": variant, "window_bufs": wb, "hash_streams": ws,
                          "windows": cnt.get("windows"), "window_pieces": cnt.get("window_pieces"),
                          "payload_bytes": cnt.get("payload_bytes"), "best_s": round(min(walls), 4),
                          "median_s": round(statistics.median(walls), 4),
                          "gbps": round(total / min(walls) / 1e9, 2), "bitfield_exact": ok,
                          **({"residency": [round(r, 4) for r in res]} if pre else {})}), flush=True)

    for b in [float(x) for x in a.budgets.split(",")]:
        budget = int(b * GiB) if b else None
        for v in (a.variants.split(",") if b else ["0:0"]):
            nb, ns = (int(x) for x in v.split(":"))
            with _context(0) as ctx:
                ctx.set_option(N.TV_OPT_WIN_BUFS, nb)
                ctx.set_option(N.TV_OPT_WIN_STREAMS, ns)
            leg("verify_payload resident", lambda: verify_payload(info, buf.mv, budget=budget, resident=True), b, v)
        # streamed: windows x columns within the budget (or 1 GiB), tv_verify_host
        leg("verify_payload streamed", lambda: verify_payload(info, buf.mv, budget=budget, resident=False), b, "columns")
    with _context(0) as ctx:
        ctx.set_option(N.TV_OPT_WIN_BUFS, 0)
        ctx.set_option(N.TV_OPT_WIN_STREAMS, 0)
    leg("verify_stream rows", lambda: verify_stream(info, lambda off, n: buf.mv[off:off + n]), None)
    buf.close()
    if a.files:   # file-backed resume under the same budgets (single16, warm page cache)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from storage_paths_bench import write_layout
        from torrent_amd import verify_files
        root = os.path.join(a.files, "single16")
        finfo, fexpect, paths = write_layout("single16", root)
        expect[:] = fexpect
        verify_files(finfo, root)          # warm the page cache and the context
        for b in [float(x) for x in a.budgets.split(",")]:
            budget = int(b * GiB) if b else None
            leg("verify_files warm", lambda: verify_files(finfo, root, budget=budget, stream=False), b, "windows")
            leg("verify_files warm streamed", lambda: verify_files(finfo, root, budget=budget, stream=True), b,
                "columns")
        if a.cold:
            import fsutil
            for b in [float(x) for x in a.budgets.split(",")]:
                budget = int(b * GiB) if b else None
                leg("verify_files cold windows", lambda: verify_files(finfo, root, budget=budget, stream=False), b,
                    "windows", pre=lambda: fsutil.drop_cache(paths))
                for v in a.cold_variants.split(","):
                    cw, cr, cq = (int(x) for x in (v + ":0:0").split(":")[:3])
                    with _context(0) as ctx:
                        ctx.set_option(N.TV_OPT_STREAM_COLD_WINDOW, cw)
                        ctx.set_option(N.TV_OPT_STREAM_COLD_READERS, cr)
                        ctx.set_option(N.TV_OPT_STREAM_COLD_REQ, cq << 10)
                    leg("verify_files cold streamed", lambda: verify_files(finfo, root, budget=budget, stream=True), b,
                        f"columns {v}", pre=lambda: fsutil.drop_cache(paths))
            with _context(0) as ctx:
                ctx.set_option(N.TV_OPT_STREAM_COLD_WINDOW, 0)
                ctx.set_option(N.TV_OPT_STREAM_COLD_READERS, 0)
                ctx.set_option(N.TV_OPT_STREAM_COLD_REQ, 0)
        for p in paths:
            os.unlink(p)


if __name__ == "__main__":
    main()
