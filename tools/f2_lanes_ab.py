"""A/B of tv_stage_files' short-segment slots on one staging lane vs alternating between two
(TV_OPT_FILE_CONCURRENT 0 / 1) on BASELINE cfg3's verify_files (10,000 files, page cache warm), interleaved
in one process: ROUNDS rounds, best of 5 calls per variant per round; every bitfield checked against the
committed one.  Then the same split for tv_stage_files alone (no verify).
usage: python tools/f2_lanes_ab.py <dir> [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.layouts import build_layout, by_name  # noqa: E402
from tests import synth  # noqa: E402
from torrent_amd import _native, verify_files  # noqa: E402
from torrent_amd.verify import _context  # noqa: E402

d = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rec = {r["name"]: r for r in json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))}["cfg3"]
lay = build_layout(by_name("cfg3"), fill=synth.fill)
info = lay["info"]
for path, data in lay["disk_files"]().items():
    p = os.path.join(d, *path)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "wb") as f:
        f.write(data)
os.chdir(d)

acc = {"stage_files": 0.0}
orig_stage = _native.Context.stage_files


def stage_files(self, *a, **k):
    t = time.perf_counter()
    r = orig_stage(self, *a, **k)
    acc["stage_files"] += time.perf_counter() - t
    return r


_native.Context.stage_files = stage_files
verify_files(info, d)  # context, ring and page cache warm
for rnd in range(rounds):
    for conc in (0, 1):
        with _context(0) as ctx:
            ctx.set_option(_native.TV_OPT_FILE_CONCURRENT, conc)
        best, best_stage = None, None
        for _ in range(5):
            acc["stage_files"] = 0.0
            t = time.perf_counter()
            bf = verify_files(info, d)
            el = time.perf_counter() - t
            assert bytes(bf).hex() == rec["expected_bitfield"]
            best = el if best is None else min(best, el)
            best_stage = acc["stage_files"] if best_stage is None else min(best_stage, acc["stage_files"])
        print(json.dumps({"round": rnd, "file_concurrent": conc, "verify_files_ms": round(best * 1e3, 2),
                          "GBps": round(info.length / best / 1e9, 2), "stage_files_ms": round(best_stage * 1e3, 2),
                          "stage_GBps": round(info.length / best_stage / 1e9, 2)}), flush=True)
