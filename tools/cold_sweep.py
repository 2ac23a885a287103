"""Cold verify_files against the box's O_DIRECT read ceiling, interleaved (is the cold path at the storage bound?).

For each layout (tools/storage_paths_bench.write_layout: single16, files64), `rounds` rounds of, each after a
residency-checked drop (tools/fsutil.drop_cache; a leg above 1 % resident is recorded and skipped):
  * the C reader's O_DIRECT ceiling at 16 threads x 4 MiB and at 64 threads x 4 MiB (tools/read_ceiling.c);
  * verify_files with O_DIRECT at 16, 32 and 64 reader threads (two staging lanes share them),
so a queue-depth effect shows beside the box's own storage variance.  Other leg sets (environment variables), each a
question the round-5 records under profiles/r05/cold_sweep_*.jsonl answer:
  COLD_LANES   one staging lane (TV_OPT_FILE_CONCURRENT = 0) against two
  COLD_DEPTH   fewer reads in flight, the library and the C reader alike
  COLD_FEW     2 and 4 reads in flight, the library on one lane
  COLD_PROBE   the C reader into page-locked buffers (RC_HOST_ALLOC_LIB) / on the GPU's NUMA node (RC_CPU_NODE);
               the library with its NUMA binding off
  COLD_SPREAD  the C reader's destination spread over 192 MiB (RC_SPREAD), as the library fills its ring
  COLD_FOOT    that destination at 16 / 32 / 48 / 64 MiB
  COLD_DMA     the C reader with a page-locked H2D DMA stream running beside it
  COLD_STRIDE  the C reader in the streamed columns' pattern (RC_STRIDE: part c of every 1 MiB piece, then c + 1)
               against sequential parts, beside verify_files windowed and streamed (0.5 GiB budget)
  COLD_LANEAB  the default bounce path (two lanes x 2 readers) against one lane x 4 readers, with the C reader
  COLD_LIBBOUNCE  the library's own bounce path (TV_OPT_FILE_BOUNCE = R readers per lane) against the ring path
               (a "verify_files" leg runs the library's default, since round 6 the bounce path with 4 readers per lane;
               "ring" names the rounds 4-5 ring path)
  COLD_BOUNCE  the C reader into its own reused buffer, then memcpy'd to the 192 MiB spread (bounce) or DMA'd to the GPU
               from two reused page-locked buffers per reader (bouncedma), against the library (round 6)

usage: python tools/cold_sweep.py <dir> [layout ...] > out.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fsutil  # noqa: E402
from storage_paths_bench import read_ceiling, write_layout  # noqa: E402
from torrent_amd import _native, verify_files  # noqa: E402
from torrent_amd.verify import _context  # noqa: E402

MiB, GiB = 1 << 20, 1 << 30


class _DmaLoad:
    """H2D DMA from a 1 GiB page-locked buffer into a resident layout, in a loop on a background thread (ctypes
    releases the GIL), as the library's staging keeps the GPU's copy engines busy beside its file reads."""

    def __init__(self):
        import threading
        self.buf = _native.PinnedBuffer(1 << 30)
        self.ctx = _native.Context(0)
        self.ctx.set_layout(4 << 30, 4 * MiB, 1024)
        self.bytes = 0
        self.halt = threading.Event()
        self.t0 = time.perf_counter()
        self.th = threading.Thread(target=self._run)
        self.th.start()

    def _run(self):
        off = 0
        while not self.halt.is_set():
            self.ctx.stage(off, self.buf.mv)
            self.bytes += 1 << 30
            off = (off + (1 << 30)) % (4 << 30)

    def stop(self):
        self.halt.set()
        self.th.join()
        g = self.bytes / (time.perf_counter() - self.t0) / 1e9
        self.ctx.close()
        self.buf.close()
        return round(g, 2)


def emit(rec):
    print(json.dumps(rec), flush=True)


def main():
    d = sys.argv[1]
    names = sys.argv[2:] or ["single16", "files64"]
    rounds = int(os.environ.get("COLD_ROUNDS", "2"))
    for name in names:
        root = os.path.join(d, name)
        info, expect, paths = write_layout(name, root)
        total = info.length
        cwd = os.getcwd()
        os.chdir(root)
        verify_files(info, root)          # context, allocations, ring (warm; not measured)
        with _context(0) as ctx:
            ctx.set_option(_native.TV_OPT_FILE_ODIRECT, 1)
        legs = [("ceiling direct 16x4MiB", 16), ("ceiling direct 64x4MiB", 64),
                ("verify_files O_DIRECT", 16), ("verify_files O_DIRECT", 32), ("verify_files O_DIRECT", 64)]
        if os.environ.get("COLD_DEPTH"):      # reads in flight: fewer threads, one or two lanes, C reader alike
            legs = [("ceiling direct 8x4MiB", 8), ("verify_files O_DIRECT", 8), ("verify_files O_DIRECT", 4),
                    ("verify_files O_DIRECT 1 lane", 8), ("ceiling direct 4x4MiB", 4), ("verify_files O_DIRECT", 12),
                    ("ceiling direct 12x4MiB", 12), ("verify_files O_DIRECT", 16)]
        if os.environ.get("COLD_PROBE"):      # what the library's reader differs in from the C reader
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 4x4MiB pinned", 4),
                    ("ceiling direct 4x4MiB node", 4), ("ceiling direct 4x4MiB pinned node", 4),
                    ("verify_files O_DIRECT 1 lane", 4), ("verify_files O_DIRECT 1 lane nobind", 4)]
        if os.environ.get("COLD_SPREAD"):     # destination footprint: a 4 MiB buffer per reader vs a 192 MiB ring
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 4x4MiB spread", 4),
                    ("ceiling direct 4x4MiB pinned spread", 4), ("verify_files O_DIRECT 1 lane", 4),
                    ("ceiling direct 16x4MiB spread", 16), ("ceiling direct 16x4MiB", 16)]
        if os.environ.get("COLD_DMA"):        # the C reader with and without the GPU's H2D DMA running beside it
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 4x4MiB dma", 4),
                    ("ceiling direct 16x4MiB", 16), ("ceiling direct 16x4MiB dma", 16),
                    ("ceiling direct 4x4MiB spread192", 4), ("ceiling direct 4x4MiB spread192 dma", 4)]
        if os.environ.get("COLD_FOOT"):       # the destination footprint at which the reads slow down
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 4x4MiB spread16", 4),
                    ("ceiling direct 4x4MiB spread32", 4), ("ceiling direct 4x4MiB spread64", 4),
                    ("ceiling direct 8x4MiB spread32", 8), ("ceiling direct 6x4MiB spread48", 6)]
        if os.environ.get("COLD_FEW"):        # few reads in flight, the library on one lane against the C reader
            legs = [("ceiling direct 4x4MiB", 4), ("verify_files O_DIRECT 1 lane", 4), ("verify_files O_DIRECT", 4),
                    ("ceiling direct 2x4MiB", 2), ("verify_files O_DIRECT 1 lane", 2), ("verify_files O_DIRECT", 16)]
        if os.environ.get("COLD_BOUNCE"):     # a compact reused read destination, then a copy or a DMA from it
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 4x4MiB spread", 4),
                    ("ceiling direct 4x4MiB bouncedma", 4), ("ceiling direct 4x4MiB bouncedma1", 4),
                    ("ceiling direct 8x4MiB bouncedma1", 8), ("ceiling direct 6x4MiB bouncedma1", 6),
                    ("verify_files O_DIRECT", 16)]
            if os.environ.get("COLD_BOUNCE") == "copy":   # (round 6's first sweep: the host-copy form too)
                legs += [("ceiling direct 4x4MiB bounce spread", 4), ("ceiling direct 8x4MiB bounce spread", 8)]
        if os.environ.get("COLD_LIBBOUNCE"):  # the library's bounce path (TV_OPT_FILE_BOUNCE readers per lane)
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 4x4MiB bouncedma1", 4),
                    ("verify_files O_DIRECT ring", 16), ("verify_files O_DIRECT bounce2", 16),
                    ("verify_files O_DIRECT bounce4", 16), ("verify_files O_DIRECT bounce2 1 lane", 16),
                    ("verify_files O_DIRECT bounce4 1 lane", 16), ("verify_files O_DIRECT bounce8", 16)]
        if os.environ.get("COLD_STRIDE"):     # the streamed columns' read pattern (RC_STRIDE) against sequential parts
            legs = [("ceiling direct 4x4MiB", 4), ("ceiling direct 16x512KiB", 16),
                    ("ceiling direct 16x512KiB stride", 16), ("ceiling direct 32x512KiB stride", 32),
                    ("ceiling direct 32x128KiB stride", 32), ("verify_files O_DIRECT bounce2", 16),
                    ("verify_files streamed 0.5GiB", 16)]
            if os.environ.get("COLD_STRIDE") == "spread":   # the same reads landing across the ring's footprint
                legs = [("ceiling direct 32x512KiB stride", 32), ("ceiling direct 32x512KiB stride spread", 32),
                        ("ceiling direct 32x512KiB stride spread48", 32), ("ceiling direct 32x512KiB stride pinned", 32),
                        ("ceiling direct 32x512KiB stride spread pinned", 32), ("verify_files streamed 0.5GiB", 16)]
        if os.environ.get("COLD_LANEAB"):     # the default (two lanes x 2 readers) against one lane x 4 readers
            legs = [("ceiling direct 4x4MiB", 4), ("verify_files O_DIRECT bounce2", 16),
                    ("verify_files O_DIRECT bounce4 1 lane", 16)]
        if os.environ.get("COLD_LANES"):      # also one staging lane (TV_OPT_FILE_CONCURRENT = 0)
            legs = [("ceiling direct 16x4MiB", 16), ("verify_files O_DIRECT", 16),
                    ("verify_files O_DIRECT 1 lane", 16), ("verify_files O_DIRECT 1 lane", 32),
                    ("ceiling direct 8x4MiB", 8), ("ceiling direct 32x4MiB", 32)]
        for rnd in range(rounds):
            for what, thr in legs:
                res = fsutil.drop_cache(paths)
                rec = {"layout": name, "round": rnd, "leg": what, "threads": thr, "resident": round(res, 4)}
                if res > 0.01:
                    rec["skipped"] = "still cached after the drop"
                    emit(rec)
                    continue
                if what.startswith("ceiling"):
                    env = {}
                    if "pinned" in what:
                        env["RC_HOST_ALLOC_LIB"] = os.path.join(ROOT, "torrent_amd", "libtorrent_verify.so")
                    if "spread" in what:
                        mib = what.split("spread", 1)[1].split()[0] if what.split("spread", 1)[1][:1].isdigit() else "192"
                        env["RC_SPREAD"] = str(int(mib) * MiB)
                    if "bouncedma" in what:
                        env["RC_BOUNCE"] = "dma1" if "bouncedma1" in what else "dma"
                    elif "bounce" in what:
                        env["RC_BOUNCE"] = "copy"
                    if "node" in what:
                        with _context(0) as ctx:
                            nd = ctx.counter(_native.TV_COUNTER_NUMA_NODE)
                        env["RC_CPU_NODE"] = str(nd if nd < (1 << 63) else 0)
                        rec["node"] = env["RC_CPU_NODE"]
                    part = 4 * MiB
                    if "KiB" in what.split("x", 1)[-1].split()[0]:   # ("ceiling direct 16x512KiB ...": 512 KiB parts)
                        part = int(what.split("x", 1)[1].split("KiB")[0]) << 10
                    if "stride" in what:   # column-major parts of 1 MiB pieces, as the streamed columns read
                        env["RC_STRIDE"] = str(MiB)
                    dma = None
                    if what.endswith(" dma"):   # (not the bouncedma legs: their DMA is the reader's own)
                        dma = _DmaLoad()
                    t = time.perf_counter()
                    try:
                        got = read_ceiling(paths, threads=thr, part=part, direct=True, env=env)
                    finally:
                        if dma:
                            rec["dma_gbps"] = dma.stop()
                    rec["gbps"] = round(got / 1e9, 2) if got else None
                    rec["s"] = round(time.perf_counter() - t, 3)
                else:
                    with _context(0) as ctx:
                        ctx._reset_file_clock()
                        ctx.set_option(_native.TV_OPT_FILE_CONCURRENT, 0 if "1 lane" in what else 1)
                        ctx.set_option(_native.TV_OPT_NUMA_BIND, 0 if "nobind" in what else 1)
                        # (bounceR: R bounce readers per lane; ring: the rounds 4-5 ring path; else the default)
                        nb = (what.split("bounce", 1)[1].split()[0] if "bounce" in what else
                              "0" if " ring" in what else str(_native.FILE_BOUNCE_DEFAULT))
                        ctx.set_option(_native.TV_OPT_FILE_BOUNCE, int(nb))
                    t = time.perf_counter()
                    bf = (verify_files(info, root, threads=thr, budget=GiB // 2, stream=True) if "streamed" in what
                          else verify_files(info, root, threads=thr))
                    el = time.perf_counter() - t
                    with _context(0) as ctx:
                        clock = ctx._file_clock()
                    rec.update({"gbps": round(total / el / 1e9, 2), "s": round(el, 3), "exact": bytes(bf) == expect,
                                "read_ms_sum_lanes": round(clock["read"] / 1e6, 1),
                                "wait_ms": round(clock["wait"] / 1e6, 1),
                                "bytes_odirect": clock["bytes_odirect"], "bytes_read": clock["bytes_read"]})
                emit(rec)
        os.chdir(cwd)
        for p in paths:
            os.unlink(p)


if __name__ == "__main__":
    main()
