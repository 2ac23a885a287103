"""Incremental-verify flush latency over the slot pool, and the CPU/GPU crossover of a short flush
(VERDICT r03 items 2 and 8).

For pieces of 256 KiB / 1 MiB / 4 MiB and flushes of n = 1 .. 4,096 pieces (4 MiB: .. 256):
  gpu_list_ms    tv_verify_list of n pieces already staged in a slot pool of 4,096 slots (the flush itself,
                 wall clock around the call; the library's kernel time beside it)
  stage_ms       staging those n pieces into their slots (paid as pieces complete, not at the flush)
  cpu_1core_ms   SHA-1 of the n pieces on one core (hashlib: OpenSSL, SHA-NI on this host -- the class of the
                 reference's WebCrypto digest; Deno's `ring` SHA-1 is software and slower, so this is the CPU's
                 best case)
  cpu_4core_ms   the same on 4 threads (Deno runs each crypto.subtle.digest on its blocking pool)
crossover_1core / _4core = the largest n for which the CPU is still faster than one GPU flush.
Every GPU result is checked against hashlib.  usage: python tools/cpu_crossover.py > out.json
"""
import hashlib
import json
import os
import statistics
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from torrent_amd import _native as N  # noqa: E402


def main():
    out = {"host_cpus_allowed": len(os.sched_getaffinity(0)), "rows": []}
    pool = ThreadPoolExecutor(4)
    for L, counts in ((256 << 10, [1, 2, 4, 8, 16, 32, 64, 256, 1024, 4096]), (1 << 20, [1, 2, 4, 8, 16, 32, 64, 256, 1024]),
                      (4 << 20, [1, 2, 4, 8, 16, 32, 64, 256])):
        P = 4096
        datas = [os.urandom(L) for _ in range(8)]            # pieces cycle through 8 random payloads
        d8 = [hashlib.sha1(x).digest() for x in datas]
        digests = b"".join(d8[i % 8] for i in range(P))
        with N.Context(0) as ctx:
            ctx.set_option(N.TV_OPT_LIST_SLOTS, min(P, max(counts)))
            ctx.set_layout(L * P, L, P)
            ctx.set_digests(bytes(digests))
            # warm-up: context, kernels, clock
            for _ in range(3):
                ctx.stage(0, datas[0])
                ctx.verify_list([0])
            rows = []
            for n in counts:
                gpu, kern, stage = [], [], []
                for rep in range(5):
                    idx = [(rep * 997 + k * 13) % P for k in range(n)]
                    idx = list(dict.fromkeys(idx))[:n]
                    t0 = time.perf_counter()
                    for i in idx:
                        ctx.stage(i * L, datas[i % 8])
                    t1 = time.perf_counter()
                    ok = ctx.verify_list(idx)
                    t2 = time.perf_counter()
                    assert all(ok), "GPU flush disagrees with hashlib"
                    gpu.append((t2 - t1) * 1e3)
                    stage.append((t1 - t0) * 1e3)
                    kern.append(ctx.last_timing()[0])
                cpu1, cpu4 = [], []
                for rep in range(3):
                    t0 = time.perf_counter()
                    for k in range(n):
                        hashlib.sha1(datas[k % 8]).digest()
                    cpu1.append((time.perf_counter() - t0) * 1e3)
                    t0 = time.perf_counter()
                    list(pool.map(lambda k: hashlib.sha1(datas[k % 8]).digest(), range(n)))
                    cpu4.append((time.perf_counter() - t0) * 1e3)
                r = {"piece_length": L, "n": n, "gpu_list_ms": round(statistics.median(gpu), 3),
                     "gpu_kernel_ms": round(statistics.median(kern), 3), "stage_ms": round(statistics.median(stage), 3),
                     "cpu_1core_ms": round(statistics.median(cpu1), 3), "cpu_4core_ms": round(statistics.median(cpu4), 3),
                     "slots_payload_bytes": ctx.counter(N.TV_COUNTER_PAYLOAD_BYTES)}
                rows.append(r)
                print(json.dumps(r), file=sys.stderr, flush=True)
            out["rows"] += rows
            for key in ("cpu_1core_ms", "cpu_4core_ms"):
                faster = [r["n"] for r in rows if r[key] < r["gpu_list_ms"]]
                out.setdefault("crossover", {})[f"{L >> 10}KiB_{key[:-3]}"] = max(faster) if faster else 0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
