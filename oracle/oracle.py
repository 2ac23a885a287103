"""ctypes binding for the CPU oracle (oracle/sha1_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, where it is the checker.  Nothing under torrent_amd/ imports it.

Parity: pinned against the reference's own fixtures (test_data/*.torrent digests, see
sha1_oracle.c header and tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_u64 = ctypes.c_uint64
_p = ctypes.c_void_p


def build() -> str:
    """Compile liboracle.so in place (gcc only)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_sha1.argtypes = [_p, _u64, _p]
        L.orc_piece_len.argtypes = [_u64, _u64, _u64, _u64]
        L.orc_piece_len.restype = _u64
        L.orc_n_pieces.argtypes = [_u64]
        L.orc_n_pieces.restype = _u64
        L.orc_verify_linear.argtypes = [_p, _u64, _u64, _p, _u64, _p, _p]
        L.orc_verify_linear.restype = _u64
        L.orc_synth_fill.argtypes = [_u64, _u64, _u64, _p]
        L.orc_synth_piece_digests.argtypes = [_u64, _u64, _u64, _u64, _u64, _u64, ctypes.c_int, _p]
        L.orc_hash_pieces.argtypes = [_p, _u64, _u64, _u64, _u64, _u64, ctypes.c_int, _p]
        L.orc_set_impl.argtypes = [ctypes.c_int]
        L.orc_set_impl.restype = ctypes.c_int
        L.orc_get_impl.restype = ctypes.c_int
        _lib = L
    return _lib


IMPL_NAMES = {1: "scalar", 2: "sha-ni"}


def set_impl(name: str) -> bool:
    """Select the compression: "best", "scalar" (plain FIPS 180-4 restatement) or "sha-ni"
    (x86 SHA extensions).  Returns False if the host lacks the requested one."""
    code = {"best": 0, "scalar": 1, "sha-ni": 2}[name]
    return lib().orc_set_impl(code) > 0


def impl() -> str:
    return IMPL_NAMES[lib().orc_get_impl()]


def _buf(b):
    """Return (ctypes pointer, keepalive) for a bytes-like object (zero-copy where possible)."""
    if b is None:
        return None, None
    if isinstance(b, bytes):
        return ctypes.cast(ctypes.c_char_p(b), _p), b
    mv = memoryview(b)
    if mv.readonly:
        bb = bytes(mv)
        return ctypes.cast(ctypes.c_char_p(bb), _p), bb
    c = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return ctypes.cast(c, _p), c


def sha1(data) -> bytes:
    out = ctypes.create_string_buffer(20)
    p, keep = _buf(data)
    lib().orc_sha1(p, len(memoryview(data).cast("B")) if not isinstance(data, bytes) else len(data), out)
    del keep
    return out.raw


def piece_len(n: int, n_pieces: int, total_length: int, piece_length: int) -> int:
    return lib().orc_piece_len(n, n_pieces, total_length, piece_length)


def verify_linear(payload, total_length: int, piece_length: int, pieces: bytes, avail=None) -> bytes:
    P = (len(pieces) + 19) // 20
    out = ctypes.create_string_buffer(max(1, (P + 7) // 8))
    pp, k1 = _buf(payload)
    dp, k2 = _buf(pieces)
    ap, k3 = _buf(avail)
    lib().orc_verify_linear(pp, total_length, piece_length, dp, len(pieces), ap, out)
    del k1, k2, k3
    return out.raw[: (P + 7) // 8]


def synth_fill(seed: int, off: int, length: int) -> bytearray:
    out = bytearray(length)
    if length:
        p, keep = _buf(out)
        lib().orc_synth_fill(seed, off, length, p)
        del keep
    return out


def synth_piece_digests(seed: int, total_length: int, piece_length: int, n_pieces: int,
                        first: int = 0, count: int | None = None, threads: int = 1) -> bytes:
    if count is None:
        count = n_pieces - first
    out = ctypes.create_string_buffer(max(1, 20 * count))
    lib().orc_synth_piece_digests(seed, total_length, piece_length, n_pieces, first, count, threads, out)
    return out.raw[: 20 * count]


def hash_pieces(payload, total_length: int, piece_length: int, n_pieces: int,
                first: int = 0, count: int | None = None, threads: int = 1) -> bytes:
    if count is None:
        count = n_pieces - first
    out = ctypes.create_string_buffer(max(1, 20 * count))
    pp, keep = _buf(payload)
    lib().orc_hash_pieces(pp, total_length, piece_length, n_pieces, first, count, threads, out)
    del keep
    return out.raw[: 20 * count]
