"""A/B of whole-call time (what the bench's `value` divides by), not kernel time: for each library variant
(build/variants/libtv_<name>.so, each in its own process, interleaved `rounds` times) the wall time per
tv_verify step at cfg2 (16,384 x 1 MiB, as bench.py's timed loop: verify + last_timing per step), its kernel
time from HIP events, and the wall time of one-piece and 64-piece tv_verify_list flushes (256 KiB pieces).

    python tools/step_ab.py <name> [<name> ...]        env: ROUNDS (3), STEPS (20)
Prints one JSON line per (variant, round)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, time, statistics
sys.path.insert(0, os.environ["TV_ROOT"])
from torrent_amd import _native as N
steps = int(os.environ.get("STEPS", "20"))
if os.environ.get("TORCH") == "1":     # as bench.py: torch imported and its device context created
    import torch
    torch.cuda.synchronize(0)
out = {}
with N.Context(0) as ctx:
    L, P = 1 << 20, 16384
    ctx.set_layout(L * P, L, P)
    ctx.fill_synthetic(2)
    d = bytearray(ctx.hash())
    d[0] ^= 1
    ctx.set_digests(bytes(d))
    for _ in range(3):
        ctx.verify()
    ks = []
    t0 = time.perf_counter()
    for _ in range(steps):
        bf = ctx.verify()
        ks.append(ctx.last_timing()[0])
    el = time.perf_counter() - t0
    assert bf[0] == 0x7F and bf[1:] == b"\xff" * (P // 8 - 1)
    out["cfg2_ms_per_step"] = round(el * 1e3 / steps, 4)
    out["cfg2_kernel_ms_avg"] = round(sum(ks) / len(ks), 4)
    out["cfg2_gap_ms"] = round(out["cfg2_ms_per_step"] - out["cfg2_kernel_ms_avg"], 4)
    L, P = 256 << 10, 4096
    ctx.set_layout(L * P, L, P)
    ctx.fill_synthetic(3)
    ctx.set_digests(ctx.hash())
    for n in (1, 64):
        lst = list(range(0, P, P // n))[:n]
        w = []
        for _ in range(steps + 2):
            t0 = time.perf_counter()
            ok = ctx.verify_list(lst)
            w.append((time.perf_counter() - t0) * 1e3)
        assert ok == b"\x01" * n
        out[f"list{n}_wall_ms_median"] = round(statistics.median(w[2:]), 4)
        out[f"list{n}_kernel_ms"] = round(ctx.last_timing()[0], 4)
print(json.dumps(out))
'''


def main():
    names = sys.argv[1:]
    for rnd in range(int(os.environ.get("ROUNDS", "3"))):
        for name in names:
            vroot = os.path.join(ROOT, "build", "variants", f"root_{name}")
            env = dict(os.environ, TV_ROOT=vroot if os.path.isdir(vroot) else ROOT,
                       TORRENT_VERIFY_LIB=os.path.join(ROOT, "build", "variants", f"libtv_{name}.so"))
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(json.dumps({"variant": name, "round": rnd, "error": r.stderr[-800:]}), flush=True)
                continue
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            rec.update(variant=name, round=rnd, torch=os.environ.get("TORCH") == "1")
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
