import os, sys, time
from concurrent.futures import ThreadPoolExecutor
sys.path.insert(0, os.getcwd())
from tests.layouts import build_layout, by_name
from tests import synth  # noqa: E402
d = "/tmp/tvfsp"
lay = build_layout(by_name("cfg3"), fill=synth.fill)
paths = []
for path, data in lay["disk_files"]().items():
    p = os.path.join(d, *path); os.makedirs(os.path.dirname(p), exist_ok=True)
    open(p, "wb").write(data); paths.append(p)
os.system(f"df -h {d} | tail -1; mount | grep -E ' /tmp | / ' | head -3")
t0 = time.perf_counter()
for p in paths:
    fd = os.open(p, os.O_RDONLY); os.close(fd)
t1 = time.perf_counter(); print(f"open+close x{len(paths)}: {(t1 - t0) * 1e6 / len(paths):.1f} us each", flush=True)
buf = bytearray(600000)
def rd(p):
    fd = os.open(p, os.O_RDONLY); n = os.readv(fd, [buf]); os.close(fd); return n
t0 = time.perf_counter(); tot = sum(rd(p) for p in paths); t1 = time.perf_counter()
print(f"1 thread read: {tot / (t1 - t0) / 1e9:.2f} GB/s", flush=True)
bufs = {}
def rd2(p):
    import threading
    b = bufs.setdefault(threading.get_ident(), bytearray(600000))
    fd = os.open(p, os.O_RDONLY); n = os.readv(fd, [b]); os.close(fd); return n
for T in (4, 16):
    with ThreadPoolExecutor(T) as ex:
        t0 = time.perf_counter(); tot = sum(ex.map(rd2, paths)); t1 = time.perf_counter()
    print(f"{T} threads read: {tot / (t1 - t0) / 1e9:.2f} GB/s", flush=True)
