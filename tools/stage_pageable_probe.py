"""Staging rate from PAGEABLE host memory (tv_stage through the pinned ring: the path of verify_payload,
hash_pieces(payload) and the Deno verifyPieces batches), with 1 vs TV_OPT_FILE_THREADS copy threads.
usage: python tools/stage_pageable_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native  # noqa: E402

L, P = 1 << 20, 4096
total = L * P
buf = bytearray(os.urandom(1 << 20) * P)
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
for threads in (1, 4, 16):
    ctx.set_option(_native.TV_OPT_FILE_THREADS, threads)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        ctx.stage(0, buf)
        best = min(best, time.perf_counter() - t0)
    print(f"tv_stage from pageable memory, {total >> 30} GiB, {threads:2d} copy threads: {total / best / 1e9:.2f} GB/s", flush=True)
ctx.close()

# the streamed path (tv_verify_host) from pageable memory: column gathers into the pinned ring
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
ctx.fill_synthetic(1)
ctx.set_digests(ctx.hash())
host = bytearray(total)
ctx.read(0, host)
for threads in (1, 16):
    ctx.set_option(_native.TV_OPT_FILE_THREADS, threads)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        bf = ctx.verify_host(host)
        best = min(best, time.perf_counter() - t0)
    assert bf == b"\xff" * (P // 8)
    print(f"tv_verify_host from pageable memory, {total >> 30} GiB, {threads:2d} copy threads: {total / best / 1e9:.2f} GB/s",
          flush=True)
ctx.close()
