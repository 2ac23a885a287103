"""Probe: can resume-from-disk skip the pread memcpy by DMA-ing straight out of the page cache?

Writes a synthetic torrent as n files, then times, per file:
  (A) verify_files (parallel preads into pinned buffers, then DMA);
  (B) mmap(PROT_READ, MAP_SHARED) + hipHostRegister(ReadOnly) + tv_stage (direct DMA) + unregister.
usage: python tools/mmap_probe.py <dir> <GiB> [n_files]"""
import ctypes
import mmap
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native, make_info, FileInfo, verify_files  # noqa: E402

d, gib = sys.argv[1], float(sys.argv[2])
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 4
L = 1 << 20
total = int(gib * (1 << 30)) // L * L
P = total // L
ctx = _native.Context(0)
ctx.set_layout(total, L, P)
ctx.fill_synthetic(5)
pieces = bytearray(ctx.hash())
for i in range(0, P, 100):
    pieces[20 * i] ^= 1
per = total // nf
sizes = [per] * (nf - 1) + [total - per * (nf - 1)]
files = [FileInfo(s, [f"f{k:04d}.bin"]) for k, s in enumerate(sizes)]
info = make_info(L, bytes(pieces), "r", files=files)
os.makedirs(d, exist_ok=True)
buf = _native.PinnedBuffer(max(sizes))
off = 0
for f in files:
    mv = buf.mv[:f.length]
    ctx.read(off, mv)
    with open(os.path.join(d, *f.path), "wb") as fh:
        fh.write(mv)
    off += f.length
buf.close()


def expect_ok(bf):
    return all(((bf[i >> 3] >> (7 - (i & 7))) & 1) == (0 if i % 100 == 0 else 1) for i in range(P))


cwd = os.getcwd()
os.chdir(d)
for rep in range(2):
    t0 = time.perf_counter()
    bf = verify_files(info, d, threads=16)
    el = time.perf_counter() - t0
    print(f"A verify_files       : {el * 1e3:7.0f} ms  {total / el / 1e9:6.2f} GB/s exact={expect_ok(bf)}", flush=True)
os.chdir(cwd)

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
libc = ctypes.CDLL(None, use_errno=True)
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
MAP_POPULATE = 0x8000

ctx.set_layout(total, L, P)
ctx.set_digests(bytes(pieces))
for flags_name, flags, mflags in (("ReadOnly", 0x08, mmap.MAP_SHARED), ("ReadOnly+POPULATE", 0x08, mmap.MAP_SHARED | MAP_POPULATE)):
    t_reg = t_stage = t_unreg = 0.0
    t0 = time.perf_counter()
    ok = True
    off = 0
    for f in files:
        fd = os.open(os.path.join(d, *f.path), os.O_RDONLY)
        addr = libc.mmap(None, f.length, mmap.PROT_READ, mflags, fd, 0)
        a = time.perf_counter()
        rc = hip.hipHostRegister(addr, f.length, flags)
        b = time.perf_counter()
        if rc != 0:
            print(f"B {flags_name}: hipHostRegister rc={rc}", flush=True)
            ok = False
            libc.munmap(addr, f.length)
            os.close(fd)
            break
        mv = memoryview((ctypes.c_char * f.length).from_address(addr)).cast("B")
        ctx.stage(off, mv)
        c = time.perf_counter()
        hip.hipHostUnregister(addr)
        e = time.perf_counter()
        libc.munmap(addr, f.length)
        os.close(fd)
        t_reg += b - a
        t_stage += c - b
        t_unreg += e - c
        off += f.length
    if not ok:
        continue
    bf = ctx.verify()
    el = time.perf_counter() - t0
    print(f"B mmap+{flags_name:18s}: {el * 1e3:7.0f} ms  {total / el / 1e9:6.2f} GB/s  (register {t_reg * 1e3:.0f} ms, "
          f"stage {t_stage * 1e3:.0f} ms = {total / t_stage / 1e9:.1f} GB/s, unregister {t_unreg * 1e3:.0f} ms) "
          f"exact={expect_ok(bf)}", flush=True)
ctx.close()
