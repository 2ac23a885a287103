"""A/B the split kernel's build variants (tools/build_variants.py) on one GPU, interleaved: for each
piece count, every variant's verify kernel time (HIP events, best and median of `reps`) on the same
synthetic payload; each variant's digests must equal the first variant's and its bitfield be exact.

    python tools/variant_bench.py <pieces,...> <name> [<name> ...]      (libs in build/variants/)
env: KERNEL (default 2 = split), PAIRS (TV_OPT_SPLIT_PAIRS, default 0), REPS (5), GIB (payload GiB per point, 16)
Each variant runs in its own process (one library per process); results as JSON lines."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, statistics
sys.path.insert(0, os.environ["TV_ROOT"])
from torrent_amd import _native as N
P = int(sys.argv[1]); reps = int(sys.argv[2]); kernel = int(sys.argv[3]); gib = int(sys.argv[4])
L = ((gib << 30) // P) // 64 * 64
ctx = N.Context(0)
ctx.set_option(N.TV_OPT_KERNEL, kernel)
ctx.set_option(N.TV_OPT_SPLIT_PAIRS, int(os.environ.get("PAIRS", "0")))
ctx.set_layout(L * P, L, P)
ctx.fill_synthetic(2)
d = bytearray(ctx.hash())
dig = bytes(d)
for i in range(0, P, 100):
    d[20 * i] ^= 1
ctx.set_digests(bytes(d))
ms = []
for _ in range(reps + 1):
    bf = ctx.verify()
    ms.append(ctx.last_timing()[0])
ms = ms[1:]
ok = all(((bf[i >> 3] >> (7 - (i & 7))) & 1) == (0 if i % 100 == 0 else 1) for i in range(P))
import hashlib
print(json.dumps({"P": P, "L": L, "best_ms": min(ms), "median_ms": statistics.median(ms), "ok": ok,
                  "digests_sha1": hashlib.sha1(dig).hexdigest(), "kernel": ctx.last_kernel()[0]}))
'''


def main():
    ps = [int(x) for x in sys.argv[1].split(",")]
    names = sys.argv[2:]
    reps = int(os.environ.get("REPS", "5"))
    kernel = int(os.environ.get("KERNEL", "2"))
    gib = int(os.environ.get("GIB", "16"))       # payload per point (GIB=200 at 51,200 pieces = cfg4)
    for P in ps:
        ref = None
        for rnd in range(2):                     # two interleaved passes over the variants
            for name in names:
                # a variant may bring its own host package (an older build's ABI): build/variants/root_<name>
                vroot = os.path.join(ROOT, "build", "variants", f"root_{name}")
                env = dict(os.environ, TV_ROOT=vroot if os.path.isdir(vroot) else ROOT,
                           TORRENT_VERIFY_LIB=os.path.join(ROOT, "build", "variants", f"libtv_{name}.so"))
                r = subprocess.run([sys.executable, "-c", CHILD, str(P), str(reps), str(kernel), str(gib)], env=env,
                                   capture_output=True, text=True, timeout=300)
                if r.returncode:
                    print(json.dumps({"variant": name, "P": P, "error": r.stderr[-800:]}), flush=True)
                    continue
                rec = json.loads(r.stdout.strip().splitlines()[-1])
                rec.update(variant=name, round=rnd, gbps=round(rec["L"] * P / rec["best_ms"] / 1e6, 1))
                ref = ref or rec["digests_sha1"]
                rec["digests_match_first"] = rec["digests_sha1"] == ref
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
