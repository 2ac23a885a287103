"""Piece-count sweep: HBM-resident verify throughput of every kernel variant vs pieces per GPU
(16 GiB payload per point, piece length = 16 GiB / P rounded to 64 B).  Substantiates the
auto kernel choice (tv_core.hip choose_kernel) and the piece-parallelism ceiling of DESIGN.md 4.
usage: python tools/sweep_pieces.py [out.jsonl]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N  # noqa: E402

VARIANTS = [("lane", 1, 0), ("split1", 2, 1), ("split2", 2, 2), ("mix", 3, 0), ("twin1", 4, 1), ("twin2", 4, 2), ("auto", 0, 0)]
if os.environ.get("SWEEP_VARIANTS"):   # e.g. lane,mix (auto is always measured last)
    VARIANTS = [v for v in VARIANTS if v[0] in os.environ["SWEEP_VARIANTS"].split(",")] + [VARIANTS[-1]]
PS = [1024, 2048, 4096, 8192, 12800, 16384, 20480, 25600, 32768, 40960, 49152, 51200, 65536, 131072, 262144]
if os.environ.get("SWEEP_PS"):
    PS = [int(x) for x in os.environ["SWEEP_PS"].split(",")]


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
    rows = []
    for P in PS:
        L = ((16 << 30) // P) // 64 * 64
        total = L * P
        ctx = N.Context(0)
        ctx.set_layout(total, L, P)
        ctx.fill_synthetic(2)
        ctx.set_option(N.TV_OPT_KERNEL, 1)
        d = bytearray(ctx.hash())
        for i in range(0, P, 100):
            d[20 * i] ^= 1
        ctx.set_digests(bytes(d))
        expect = [0 if i % 100 == 0 else 1 for i in range(P)]
        row = {"pieces": P, "piece_length": L, "bytes": total}
        for name, k, pairs in VARIANTS:
            ctx.set_option(N.TV_OPT_KERNEL, k)
            ctx.set_option(N.TV_OPT_SPLIT_PAIRS, pairs)
            best = 1e9
            for _ in range(3):
                bf = ctx.verify()
                best = min(best, ctx.last_timing()[0])
            bits = [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)]
            assert bits == expect, (P, name)
            row[name] = round(total / best / 1e6, 1)   # GB/s
            ctx.set_digests(bytes(len(d)))             # all-zero digests: every bit must now read 0
            assert not any(ctx.verify()), (P, name)    # (no stale bits from the previous variant)
            ctx.set_digests(bytes(d))
            if name == "auto":
                row["auto_kernel"] = {1: "lane", 2: "split", 3: "mix", 4: "twin"}[ctx.last_kernel()[0]]
        ctx.close()
        row["best"] = max((row[n], n) for n, _, _ in VARIANTS[:-1])[1]
        rows.append(row)
        line = json.dumps(row)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()
    names = [n for n, _, _ in VARIANTS]
    print("| pieces | piece length | " + " | ".join(names) + " |")
    print("|---|---|" + "---|" * len(names))
    for r in rows:
        cells = [f"{r[n]:,}" + (f" ({r['auto_kernel']})" if n == "auto" else "") for n in names]
        print(f"| {r['pieces']:,} | {r['piece_length']:,} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
