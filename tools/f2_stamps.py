"""Stamped breakdown of verify_files on warm 16 GiB layouts.

For each layout (single16: one 16 GiB file; files64: 16 GiB in 64 files; 1 MiB pieces, 1 % corrupted, hashlib's
bits; written by tools/storage_paths_bench.write_layout) and each file-staging configuration of the library
(TV_OPT_FILE_DIRECT: registered page-cache DMA vs preads into the pinned ring; TV_OPT_FILE_CONCURRENT: one or two
staging lanes; reader threads), verify_files runs `reps` times on a warm page cache (residency measured by mincore
before every leg), and the line gives the best wall time, its GB/s, exactness, and the library's file-staging phase
clock of that call (tv_options_internal.h TV_FILE_PHASE_*: ns summed over the lanes, and per 256 MiB of payload),
plus the parts of the call outside tv_stage_files (layout + digests before, the verify kernel after).

usage: python tools/f2_stamps.py <dir> [layout ...] > out.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fsutil  # noqa: E402
from storage_paths_bench import write_layout  # noqa: E402
from torrent_amd import _native, verify_files  # noqa: E402
from torrent_amd.verify import _context  # noqa: E402

MiB, GiB = 1 << 20, 1 << 30
FILE_DIRECT, FILE_CHUNK, FILE_CONCURRENT = _native.TV_OPT_FILE_DIRECT, _native.TV_OPT_FILE_CHUNK, _native.TV_OPT_FILE_CONCURRENT

CFG3_CONFIGS = [  # 10,000 files of <= 512 KiB: every segment takes the short-segment path
    ("short segments, 1 lane, 16 thr", 0, 0, 16, 256 * MiB),
    ("short segments, 2 lanes, 16 thr", 0, 1, 16, 256 * MiB),
    ("short segments, 2 lanes, 8 thr", 0, 1, 8, 256 * MiB),
    ("short segments, 2 lanes, 32 thr", 0, 1, 32, 256 * MiB),
]
COLD_CONFIGS = [  # after fsutil.drop_cache (residency re-checked): (name, odirect)
    ("cold, pread 2 lanes 16 thr, O_DIRECT", 1),
    ("cold, pread 2 lanes 16 thr, buffered", 0),
]
CONFIGS = [  # name, direct, concurrent, threads, chunk
    ("direct, 1 lane", 1, 0, 16, 256 * MiB),
    ("direct, 2 lanes", 1, 1, 16, 256 * MiB),
    ("pread, 1 lane, 16 thr", 0, 0, 16, 256 * MiB),
    ("pread, 2 lanes, 16 thr", 0, 1, 16, 256 * MiB),
    ("pread, 2 lanes, 8 thr", 0, 1, 8, 256 * MiB),
    ("pread, 2 lanes, 4 thr", 0, 1, 4, 256 * MiB),
    ("pread, 2 lanes, 16 thr, 64 MiB units", 0, 1, 16, 64 * MiB),
]


def emit(rec):
    print(json.dumps(rec), flush=True)


def main():
    d = sys.argv[1]
    names = sys.argv[2:] or ["single16", "files64", "cfg3"]
    reps = int(os.environ.get("F2_REPS", "3"))
    emit({"host": {"cpus_allowed": len(os.sched_getaffinity(0))}})
    for name in names:
        root = os.path.join(d, name)
        t0 = time.perf_counter()
        info, expect, paths = write_layout(name, root)
        cwd = os.getcwd()
        os.chdir(root)       # (Storage paths are relative to the working directory, storage.ts)
        total = info.length
        emit({"layout": name, "files": len(paths), "bytes": total, "pieces": info.n_pieces,
              "write_s": round(time.perf_counter() - t0, 1)})
        verify_files(info, root)            # context creation, allocations, first touch of the ring
        for cname, direct, conc, threads, chunk in (CFG3_CONFIGS if name == "cfg3" else CONFIGS):
            with _context(0) as ctx:
                ctx.set_option(FILE_DIRECT, direct)
                ctx.set_option(FILE_CONCURRENT, conc)
                ctx.set_option(FILE_CHUNK, chunk)
            best = None
            for _ in range(reps):
                res = fsutil.resident(paths)
                with _context(0) as ctx:
                    ctx._reset_file_clock()
                t = time.perf_counter()
                bf = verify_files(info, root, threads=threads)
                el = time.perf_counter() - t
                with _context(0) as ctx:
                    clock = ctx._file_clock()
                    kms, tms = ctx.last_timing()
                if best is None or el < best[0]:
                    best = (el, bytes(bf) == expect, clock, res, kms)
            el, exact, clock, res, kms = best
            per = total / (256 * MiB)
            emit({"layout": name, "config": cname, "direct": direct, "concurrent": conc, "threads": threads,
                  "chunk_mib": chunk // MiB, "resident": round(res, 4), "best_s": round(el, 4),
                  "gbps": round(total / el / 1e9, 2), "exact": exact,
                  "stage_files_ms": round(clock["call"] / 1e6, 1),
                  "outside_stage_files_ms": round(el * 1e3 - clock["call"] / 1e6, 1),
                  "verify_kernel_ms": round(kms, 2),
                  "phase_ms": {ph: round(v / 1e6, 1) for ph, v in clock.items() if not ph.startswith("bytes")},
                  "phase_ms_per_256MiB": {ph: round(v / 1e6 / per, 3) for ph, v in clock.items()
                                          if not ph.startswith("bytes") and ph != "call"},
                  "bytes_direct": clock["bytes_direct"], "bytes_read": clock["bytes_read"],
                  "bytes_odirect": clock["bytes_odirect"]})
        if os.environ.get("F2_COLD", "1") == "1" and name != "cfg3":
            for cname, odirect in COLD_CONFIGS:
                with _context(0) as ctx:
                    ctx.set_option(FILE_DIRECT, 0)
                    ctx.set_option(FILE_CONCURRENT, 1)
                    ctx.set_option(FILE_CHUNK, 256 * MiB)
                    ctx.set_option(_native.TV_OPT_FILE_ODIRECT, odirect)
                    ctx._reset_file_clock()
                res = fsutil.drop_cache(paths)
                t = time.perf_counter()
                bf = verify_files(info, root)
                el = time.perf_counter() - t
                with _context(0) as ctx:
                    clock = ctx._file_clock()
                    ctx.set_option(_native.TV_OPT_FILE_ODIRECT, 1)
                emit({"layout": name, "config": cname, "resident": round(res, 4), "best_s": round(el, 4),
                      "gbps": round(total / el / 1e9, 2), "exact": bytes(bf) == expect,
                      "stage_files_ms": round(clock["call"] / 1e6, 1),
                      "phase_ms": {ph: round(v / 1e6, 1) for ph, v in clock.items() if not ph.startswith("bytes")},
                      "bytes_read": clock["bytes_read"], "bytes_odirect": clock["bytes_odirect"]})
        with _context(0) as ctx:   # back to the library defaults
            ctx.set_option(FILE_DIRECT, 0)
            ctx.set_option(FILE_CONCURRENT, 1)
            ctx.set_option(FILE_CHUNK, 256 * MiB)
        os.chdir(cwd)
        for p in paths:
            os.unlink(p)


if __name__ == "__main__":
    main()
