"""The library's host-side synthetic producer (tv_host.cpp: tv_synth_fill_host, behind tv_stream_fill_synthetic)
against the oracle's synthetic bytes, on the CPU: the source is compiled with the host compiler into a small
harness (the same flags as the library build), covering the scalar head/tail, the AVX-512 store path and the
non-temporal path (fills >= 64 KiB) at unaligned offsets and destinations; and tv_copy_host, the ring-slot
copy, byte-exact at any alignment with nothing written past the end."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "torrent_amd", "csrc", "tv_host.cpp")


@pytest.fixture(scope="module")
def gen(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("hostgen") / "libhostgen.so")
    subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", SRC, "-o", so])
    lib = ctypes.CDLL(so)
    fn = lib._Z18tv_synth_fill_hostmmmPh
    fn.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    fn.restype = None
    fn._so = so
    return fn


@pytest.mark.parametrize("seed,off,n,dst_skew", [
    (1, 0, 0, 0), (1, 3, 5, 1), (7, 0, 4096, 0), (7, 5, 4099, 3),
    (9, 0, 1 << 16, 0),                 # exactly the non-temporal threshold, aligned
    (9, 8 * 12345 + 3, (1 << 18) + 17, 5),   # unaligned offset, destination and length
    (2, (4 << 20) * 51199, 256 << 10, 0),    # a cfg5 column row at the torrent's last piece
])
def test_host_generator_matches_oracle(gen, oracle, seed, off, n, dst_skew):
    buf = (ctypes.c_uint8 * (n + 128))()
    base = ctypes.addressof(buf)
    dst = base + ((-base) % 64) + dst_skew
    gen(seed, off, n, dst)
    got = ctypes.string_at(dst, n)
    assert got == bytes(oracle.synth_fill(seed, off, n))


@pytest.mark.parametrize("n,src_skew,dst_skew", [(0, 0, 0), (100, 3, 1), ((64 << 10) - 1, 0, 0), (64 << 10, 0, 0),
                                                 ((1 << 20) + 77, 5, 13), ((4 << 20) + 3, 63, 1)])
def test_host_copy_exact(gen, n, src_skew, dst_skew):
    """tv_copy_host (ring-slot copies; non-temporal at >= 64 KiB) copies every byte, at any alignment."""
    lib = ctypes.CDLL(gen._so)
    cp = lib._Z12tv_copy_hostPhPKhm
    cp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    src = os.urandom(n + 128)
    sb = ctypes.create_string_buffer(src, len(src))
    db = (ctypes.c_uint8 * (n + 128))()
    sa, da = ctypes.addressof(sb), ctypes.addressof(db)
    s0 = sa + ((-sa) % 64) + src_skew
    d0 = da + ((-da) % 64) + dst_skew
    ctypes.memset(da, 0xAB, n + 128)
    cp(d0, s0, n)
    assert ctypes.string_at(d0, n) == ctypes.string_at(s0, n)
    assert ctypes.string_at(d0 + n, (da + n + 128) - (d0 + n)) == b"\xab" * ((da + n + 128) - (d0 + n))
