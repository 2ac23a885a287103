"""Interleaved A/B of library builds on BASELINE cfg3's verify_files (10,000 files, page cache warm): each
variant (build/variants/libtv_<name>.so) in its own process, three interleaved rounds, best of 5 calls per
process; every bitfield checked against the committed one.  Also prints where the process may run (CPUs,
NUMA nodes) and the GPU's NUMA node, since the reader threads copy page-cache bytes into pinned memory.
    python tools/f2_ab.py <dir> <name>[@<cpus>] ...      e.g. f2base f2base@0-63,128-191 f2base@64-127,192-255"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import json, os, sys, time
if os.environ.get("CPUS"):                      # before anything touches the GPU: threads and pinned pages
    lo_hi = [tuple(map(int, r.split("-"))) for r in os.environ["CPUS"].split(",")]
    os.sched_setaffinity(0, {c for a, b in lo_hi for c in range(a, b + 1)})
sys.path.insert(0, os.environ["TV_ROOT"])
from tests.layouts import build_layout, by_name
from tests import synth  # noqa: E402
from torrent_amd import verify_files
d = sys.argv[1]
rec = {r["name"]: r for r in json.load(open(os.path.join(os.environ["TV_ROOT"], "tests", "golden", "layouts.json")))}["cfg3"]
info = build_layout(by_name("cfg3"), fill=synth.fill)["info"]
os.chdir(d)
best = None
for _ in range(5):
    t = time.perf_counter()
    bf = verify_files(info, d)
    el = time.perf_counter() - t
    assert bytes(bf).hex() == rec["expected_bitfield"]
    best = el if best is None else min(best, el)
import ctypes
from torrent_amd import _native
buf = ctypes.create_string_buffer(64)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipDeviceGetPCIBusId(buf, 64, 0)
bdf = buf.value.decode().lower()
try:
    node = open(f"/sys/bus/pci/devices/{bdf}/numa_node").read().strip()
except OSError:
    node = "?"
nodes = {}
try:
    from torrent_amd.verify import _context
    with _context(0) as ctx:
        nodes = {"ctx_numa_node": ctx.counter(_native.TV_COUNTER_NUMA_NODE),
                 "ring_node": ctx.counter(_native.TV_COUNTER_RING_NODE)}
except Exception as e:  # an older library without these counters
    nodes = {"counters": str(e)[:80]}
print(json.dumps(dict({"best_ms": round(best * 1e3, 2), "GBps": round(info.length / best / 1e9, 2), "gpu_bdf": bdf,
                       "gpu_node": node}, **nodes)))
'''


def numa_info():
    out = {}
    try:
        for line in open("/proc/self/status"):
            if line.startswith(("Cpus_allowed_list", "Mems_allowed_list")):
                k, v = line.split(":", 1)
                out[k] = v.strip()
    except OSError:
        pass
    nodes = {}
    base = "/sys/devices/system/node"
    if os.path.isdir(base):
        for n in sorted(os.listdir(base)):
            if n.startswith("node"):
                try:
                    nodes[n] = open(os.path.join(base, n, "cpulist")).read().strip()
                except OSError:
                    pass
    out["nodes"] = nodes
    gpus = []
    drm = "/sys/class/drm"
    if os.path.isdir(drm):
        for card in sorted(os.listdir(drm)):
            p = os.path.join(drm, card, "device", "numa_node")
            if card.startswith("card") and "-" not in card and os.path.exists(p):
                gpus.append({card: open(p).read().strip()})
    out["gpu_numa_nodes"] = gpus
    return out


def main():
    d, names = sys.argv[1], sys.argv[2:]
    from tests.layouts import build_layout, by_name
    lay = build_layout(by_name("cfg3"), fill=synth.fill)
    for path, data in lay["disk_files"]().items():
        p = os.path.join(d, *path)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(data)
    print(json.dumps({"placement": numa_info()}), flush=True)
    # a variant is <lib>[@<cpu list>]: the library build, and optionally the CPUs the process is confined to
    for rnd in range(int(os.environ.get("ROUNDS", "3"))):
        for spec in names:
            name, _, cpus = spec.partition("@")
            env = dict(os.environ, TV_ROOT=ROOT, CPUS=cpus,
                       TORRENT_VERIFY_LIB=os.path.join(ROOT, "build", "variants", f"libtv_{name}.so"))
            r = subprocess.run([sys.executable, "-c", CHILD, d], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(json.dumps({"variant": name, "round": rnd, "error": r.stderr[-600:]}), flush=True)
                sys.exit(1)
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            rec.update(variant=spec, round=rnd)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
