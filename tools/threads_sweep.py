"""verify_pieces / verify_stream over Storage(fs_storage) by reader threads (1 .. 16), page cache warm: how many
threads the reference-shaped Storage paths should use per layout.  Every bitfield is checked against the committed /
hashlib bits (tools/storage_paths_bench.write_layout).

    THREADS=1,2,4,8,16 REPS=2 python tools/threads_sweep.py DIR [cfg3|single16|files64 ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from storage_paths_bench import write_layout  # noqa: E402
from torrent_amd import Storage, fs_storage, verify_pieces, verify_stream  # noqa: E402


THREADS = [int(x) for x in os.environ.get("THREADS", "1,2,4,8,16").split(",")]
REPS = int(os.environ.get("REPS", "2"))


def main():
    d = sys.argv[1]
    for layout in sys.argv[2:] or ["cfg3"]:
        root = os.path.join(d, layout)
        info, expect, _ = write_layout(layout, root)
        cwd = os.getcwd()
        os.chdir(root)
        try:
            st = Storage(fs_storage, info, root)
            for path, fn in (("verify_pieces", lambda t: verify_pieces(info, st, threads=t)),
                             ("verify_stream rows", lambda t: verify_stream(info, st.get, threads=t))):
                for t in THREADS:
                    best, ok = None, True
                    for _ in range(REPS):
                        t0 = time.perf_counter()
                        bf = fn(t)
                        el = time.perf_counter() - t0
                        ok &= bytes(bf) == bytes(expect)
                        best = el if best is None else min(best, el)
                    print(json.dumps({"layout": layout, "path": path, "threads": t, "best_s": round(best, 4),
                                      "gbps": round(info.length / best / 1e9, 2), "exact": ok}), flush=True)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
