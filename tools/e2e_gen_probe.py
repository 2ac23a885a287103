"""Generator-fed stream (tv_stream_* + tv_stream_fill_synthetic) against generator threads: 12,800 x 4 MiB
pieces (50 GiB, one cfg5 shard at N=4) through the 3 x 64 MiB ring, 256 KiB columns; GB/s and the
producer's time in tv_stream_next (waiting for a free slot) vs fill + commit.  usage: python
tools/e2e_gen_probe.py [threads,...] [pageable]
pageable: the rows are copied by the library (tv_stream_commit_from -> pool threads) from a 1 GiB pageable
buffer of 256 pieces instead of generated.  TORRENT_VERIFY_NT_STORES=0 turns the non-temporal stores off."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N  # noqa: E402


def main():
    ths = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,8,12,16").split(",")]
    pageable = len(sys.argv) > 2 and sys.argv[2] == "pageable"
    L, P = 4 << 20, 12800
    pool = bytearray(os.urandom(1 << 20)) * 1024 if pageable else None   # 1 GiB, 256 pieces
    with N.Context(0) as ctx:
        ctx.set_option(N.TV_OPT_RESIDENT, 0)
        ctx.set_option(N.TV_OPT_STREAM_CHUNK, 256 << 10)
        ctx.set_layout(L * P, L, P)
        ctx.set_digests(bytes(20 * P))
        for th in ths + ths[:1]:
            ctx.set_option(N.TV_OPT_FILE_THREADS, th)
            nxt = fill = 0.0
            t0 = time.perf_counter()
            ctx.stream_begin()
            while True:
                a = time.perf_counter()
                req = ctx.stream_next()
                b = time.perf_counter()
                nxt += b - a
                if not req.rows:
                    break
                if pageable:
                    ctx.stream_commit_from(req, pool, L, (req.piece % 256) * L + req.offset)
                else:
                    ctx.stream_fill_synthetic(req, 4)
                    ctx.stream_commit(req)
                fill += time.perf_counter() - b
            ctx.stream_end()
            el = time.perf_counter() - t0
            print(json.dumps({"mode": "pageable" if pageable else "generated",
                              "nt_stores": os.environ.get("TORRENT_VERIFY_NT_STORES", "1"), "threads": th, "GBps": round(L * P / el / 1e9, 2), "next_s": round(nxt, 3),
                              "fill_commit_s": round(fill, 3)}), flush=True)


if __name__ == "__main__":
    main()
