"""Does NUMA placement matter for the streamed (cfg5) path?  On one GPU of a two-socket node:

  * the device's closest host NUMA node (hipDeviceAttributeHostNumaId);
  * where hipHostMalloc'd pages land (move_pages(2) query) when the allocating thread runs on the device's
    node vs the other node;
  * the generator-fed stream (tv_stream_fill_synthetic -> ring slot -> PCIe -> lane kernel) with the calling
    thread and the library's worker pool pinned to the local node vs the remote node.

    python tools/numa_probe.py [pieces]        (default 25,600 x 4 MiB = 100 GiB per pass)
Each placement runs in its own process (the affinity is set before the context and its ring exist).
Prints one JSON line per placement."""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SYS_move_pages = 279


def node_cpus(node: int) -> list:
    txt = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    out = []
    for part in txt.split(","):
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def page_nodes(ptr: int, nbytes: int, samples: int = 64) -> dict:
    libc = ctypes.CDLL(None, use_errno=True)
    step = max(4096, (nbytes // samples) // 4096 * 4096)
    addrs = [ptr + k * step for k in range(min(samples, nbytes // step))]
    pages = (ctypes.c_void_p * len(addrs))(*addrs)
    status = (ctypes.c_int * len(addrs))()
    rc = libc.syscall(SYS_move_pages, 0, len(addrs), pages, None, status, 0)
    if rc != 0:
        return {"error": os.strerror(ctypes.get_errno())}
    hist = {}
    for s in status:
        hist[str(s)] = hist.get(str(s), 0) + 1
    return hist


def host_numa_id(device: int = 0) -> int:
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    v = ctypes.c_int(-1)
    attr = None
    # hipDeviceAttributeHostNumaId's enum value differs across ROCm releases: find it by name in the header
    hdr = open("/opt/rocm/include/hip/hip_runtime_api.h").read()
    start = hdr.index("typedef enum hipDeviceAttribute_t")
    body = hdr[start:hdr.index("} hipDeviceAttribute_t", start)]
    val = -1
    for line in body.splitlines():
        line = line.split("//")[0].strip().rstrip(",")
        if not line.startswith("hipDeviceAttribute"):
            continue
        name, _, rhs = line.partition("=")
        val = int(rhs.strip(), 0) if rhs.strip() else val + 1
        if name.strip() == "hipDeviceAttributeHostNumaId":
            attr = val
            break
    if attr is not None and hip.hipDeviceGetAttribute(ctypes.byref(v), attr, device) == 0 and v.value >= 0:
        return v.value
    # fallback: the PCI device's numa_node in sysfs
    bus = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(bus, 64, device) == 0:
        path = f"/sys/bus/pci/devices/{bus.value.decode().lower()}/numa_node"
        if os.path.exists(path):
            return int(open(path).read())
    return -1


CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.environ["TV_ROOT"])
cpus = [int(x) for x in os.environ["PROBE_CPUS"].split(",")]
os.sched_setaffinity(0, cpus)
from tools.numa_probe import page_nodes
from torrent_amd import _native as N
P = int(sys.argv[1]); L = 4 << 20
buf = N.PinnedBuffer(64 << 20)
buf.mv[::4096] = bytes(len(buf.mv[::4096]))
alloc_nodes = page_nodes(buf.ptr, buf.nbytes)
buf.close()
ctx = N.Context(0)
ctx.set_option(N.TV_OPT_RESIDENT, 0)
ctx.set_option(N.TV_OPT_STREAM_CHUNK, 256 << 10)
ctx.set_option(N.TV_OPT_FILE_THREADS, 8)
ctx.set_layout(L * P, L, P)
ctx.set_digests(bytes(20 * P))
def run():
    ctx.stream_begin()
    n = 0
    while True:
        req = ctx.stream_next()
        if not req.rows:
            break
        ctx.stream_fill_synthetic(req, 4)
        ctx.stream_commit(req)
        n += 1
    return ctx.stream_end(), n
ctx.stream_begin(); r = ctx.stream_next(); ctx.stream_fill_synthetic(r, 4); ctx.stream_commit(r); ctx.stream_abort()
best = 0.0
for _ in range(2):
    t0 = time.perf_counter(); bf, n = run(); el = time.perf_counter() - t0
    best = max(best, L * P / el / 1e9)
print(json.dumps({"gbps": round(best, 2), "requests": n, "pinned_alloc_page_nodes": alloc_nodes}))
ctx.close()
'''


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 25600
    # asked in a child: this process never initialises the GPU (it only starts children)
    r = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); "
                        "from tools.numa_probe import host_numa_id; print(host_numa_id(0))" % ROOT],
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    local = int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else -1
    if local < 0:
        print(json.dumps({"host_numa_id_error": (r.stdout + r.stderr)[-600:]}), flush=True)
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
    allowed = set(os.sched_getaffinity(0))
    print(json.dumps({"device0_host_numa_id": local, "nodes": nodes, "allowed_cpus": len(allowed)}), flush=True)
    if local < 0 or len(nodes) < 2:
        return 0
    remote = [n for n in nodes if n != local][0]
    for rnd in range(2):
        for name, node in (("local", local), ("remote", remote)):
            cpus = [c for c in node_cpus(node) if c in allowed][:16]
            env = dict(os.environ, TV_ROOT=ROOT, PROBE_CPUS=",".join(map(str, cpus)))
            t0 = time.time()
            r = subprocess.run([sys.executable, "-c", CHILD, str(P)], env=env, capture_output=True, text=True,
                               timeout=300, cwd=ROOT)
            rec = {"placement": name, "node": node, "round": rnd, "wall_s": round(time.time() - t0, 1)}
            if r.returncode:
                rec["error"] = r.stderr[-600:]
            else:
                rec.update(json.loads(r.stdout.strip().splitlines()[-1]))
            print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
