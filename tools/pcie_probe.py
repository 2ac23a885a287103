"""The ceilings e2e_cfg5 is measured against, on the GPU box: host -> HBM DMA of one large page-locked
buffer (hipMemcpyAsync through torch, and the library's own 2D column copies via tv_stream_commit_from),
pageable -> HBM, and the host generator alone (tv_stream_fill_synthetic re-filling one 64 MiB ring slot on
the box's allowed cores).  usage: python tools/pcie_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N  # noqa: E402


def main():
    import bench
    import torch
    out = {"cores": bench.cpu_share()["cores"]}
    n = 1 << 30
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for name, pin in (("pinned", True), ("pageable", False)):
        h = torch.empty(n, dtype=torch.uint8, pin_memory=pin)
        h.fill_(7)
        dev.copy_(h, non_blocking=pin)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            dev.copy_(h, non_blocking=pin)
        torch.cuda.synchronize()
        out[f"h2d_{name}_1GiB_GBps"] = round(5 * n / (time.perf_counter() - t0) / 1e9, 2)
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        h.copy_(dev, non_blocking=True)
    torch.cuda.synchronize()
    out["d2h_pinned_1GiB_GBps"] = round(5 * n / (time.perf_counter() - t0) / 1e9, 2)
    del dev, h
    # the host generator alone: re-fill one lent 64 MiB slot (4 MiB pieces, 256 KiB columns)
    L, P = 4 << 20, 6400
    with N.Context(0) as ctx:
        ctx.set_option(N.TV_OPT_RESIDENT, 0)
        ctx.set_option(N.TV_OPT_STREAM_CHUNK, 256 << 10)
        for threads in sorted({1, out["cores"] // 2, out["cores"]}):
            ctx.set_option(N.TV_OPT_FILE_THREADS, max(1, threads))
            ctx.set_layout(L * P, L, P)
            ctx.set_digests(bytes(20 * P))
            ctx.stream_begin()
            req = ctx.stream_next()
            ctx.stream_fill_synthetic(req, 4)
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 1.0:
                ctx.stream_fill_synthetic(req, 4)
                reps += 1
            el = time.perf_counter() - t0
            out[f"generator_{threads}_threads_GBps"] = round(reps * req.rows * req.width / el / 1e9, 2)
            ctx.stream_abort()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
