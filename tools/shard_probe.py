"""One GPU running ONE rank's shard of a strong-scaled torrent (BASELINE cfg4 at N = 2/4/8 by default): the
exact per-GPU geometry the driver's multi-GPU bench gives each rank, for rocprofv3 kernel traces and PMC passes.

    python tools/shard_probe.py [--pieces 51200] [--piece-mib 4] [--shards 2] [--rank 0]
                                [--kernel 0] [--twin-fill 1] [--fill-reads 0] [--reps 5] [--warmup 2]

Fills the shard with the synthetic payload on the device, hashes it (creation mode) to get the digests,
corrupts 1 %, then times `reps` verify calls (HIP events on the library's stream) and checks every bit.
Prints one JSON line: kernel, workgroups, kernel ms per call, GB/s, piece ceiling share."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from torrent_amd import _native as N  # noqa: E402
from torrent_amd.verify import shard_ranges  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=51200)
    ap.add_argument("--piece-mib", type=int, default=4)
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--twin-fill", type=int, default=1)
    ap.add_argument("--fill-reads", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    L = a.piece_mib << 20
    P = a.pieces
    first, count = shard_ranges(P, a.shards)[a.rank]
    with N.Context(0) as ctx:
        ctx.set_option(N.TV_OPT_KERNEL, a.kernel)
        ctx.set_option(N.TV_OPT_TWIN_FILL, a.twin_fill)
        ctx.set_option(N.TV_OPT_TWIN_FILL_READS, a.fill_reads)
        ctx.set_layout(L * P, L, P, first, count)
        ctx.fill_synthetic(4)
        dig = bytearray(ctx.hash())
        bad = set(range(3, count, 100))
        for j in bad:
            dig[20 * j + 5] ^= 0x08
        pieces = bytearray(20 * P)
        pieces[20 * first:20 * (first + count)] = dig
        ctx.set_digests(bytes(pieces))
        ms = []
        for k in range(a.warmup + a.reps):
            bf = ctx.verify()
            if k >= a.warmup:
                ms.append(ctx.last_timing()[0])
        exact = all(((bf[j >> 3] >> (7 - (j & 7))) & 1) == (0 if j in bad else 1) for j in range(count))
        kernel = ctx.last_kernel()[0]
        wgs = ctx.counter(N.TV_COUNTER_LAST_WORKGROUPS)
    avg = sum(ms) / len(ms)
    gbps = L * count / (avg / 1e3) / 1e9
    ceil = bench.piece_ceiling(kernel, count)
    print(json.dumps({"pieces_per_gpu": count, "piece_length": L, "shard": [first, count], "shards": a.shards,
                      "kernel": bench.KERNEL_NAMES.get(kernel, kernel), "twin_fill": a.twin_fill, "fill_reads": a.fill_reads, "workgroups": wgs,
                      "kernel_ms": [round(x, 3) for x in ms], "kernel_ms_avg": round(avg, 3),
                      "kernel_ms_median": round(statistics.median(ms), 3), "gbps": round(gbps, 1),
                      "piece_ceiling_gbps": round(ceil, 1), "frac_of_piece_ceiling": round(gbps / ceil, 4),
                      "bitfield_exact": exact}), flush=True)
    return 0 if exact else 1


if __name__ == "__main__":
    sys.exit(main())
