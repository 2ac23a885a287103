#!/usr/bin/env python3
"""Generate torrent_amd/csrc/sha1_asm.h: gfx950 inline-asm SHA-1 compression blocks.

Why generated asm: hipcc (ROCm 7.2) does not fold XOR3 / Maj into v_bitop3_b32 (one
compression compiles to ~790 VALU instead of ~613), and it pads every inline-asm boundary
with `s_nop 0`, which costs a full issue slot for a lone wave.  So each compression is ONE
asm statement, and this script emits it.  The emitted instruction stream is executed by the
emulator below against hashlib before the header is written (`--check`, also run by
tests/test_asm_gen.py), so a wrong register rotation can never reach the GPU.

Blocks emitted
--------------
SHA1_FULL   one 64-byte block, message schedule computed in-asm (16-word rolling window).
            5 VALU per round + 3 per scheduled word = 400 + 192 = 592 (+16 v_perm bswap and
            5 feed-forward adds by the compiler outside) = 613 per block.
SHA1_LDS    the 80 rounds only (400 VALU); W[0..79] comes from LDS as 20 ds_read_b128
            (layout [t/4][lane][4 words], conflict-free), kept 3 quads ahead in a 16-VGPR
            ring of PHYSICAL registers (a 128-bit asm operand cannot be split in AMDGPU asm).

Round (roles rotate statically; the new `a` is written into the old `e` register):
    E  = v_add3_u32(E, K, W[t])          # off the critical path
    T0 = v_alignbit_b32(A, A, 27)        # rotl5(a)
    T1 = f(B, C, D)                      # v_bfi_b32 (Ch) | v_bitop3_b32 0x96 (Parity) / 0xE8 (Maj)
    B  = v_alignbit_b32(B, B, 2)         # rotl30(b)
    E  = v_add3_u32(E, T0, T1)           # new a
Chaining values H are read-only inputs: the first write to each working register goes to its
R output instead (no per-block v_mov), and the caller adds H += R afterwards.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import struct
import sys

K = [0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xCA62C1D6]
M32 = 0xFFFFFFFF

# physical VGPRs used by SHA1_LDS for its W ring (4 quads, 16-aligned is not required,
# quad-aligned is).  The kernel's VGPR count is therefore >= RING_BASE + 16.
RING_BASE = 64
RING_QUADS = 4


def f_kind(t: int) -> str:
    if t < 20:
        return "ch"
    if t < 40 or t >= 60:
        return "par"
    return "maj"


class Regs:
    """Map logical state slots 0..4 to asm operand names with the first-write redirect."""

    def __init__(self):
        self.cur = [f"h{i}" for i in range(5)]

    def rd(self, s: int) -> str:
        return self.cur[s]

    def wr(self, s: int) -> str:
        self.cur[s] = f"r{s}"
        return self.cur[s]


def roles(t: int):
    m = t % 5
    return [(0 - m) % 5, (1 - m) % 5, (2 - m) % 5, (3 - m) % 5, (4 - m) % 5]


def _fop(t, dst, b, c, d):
    k = f_kind(t)
    if k == "ch":
        return ("v_bfi_b32", dst, b, c, d)
    return ("v_bitop3_b32", dst, b, c, d, 0x96 if k == "par" else 0xE8)


def gen_full():
    """SHA1_FULL instruction list. Operands: r0-4 (out), w0-15 (in/out), t0-2 (tmp),
    h0-4 (in), k0-3 (sgpr in)."""
    ins = []
    R = Regs()
    for t in range(80):
        A, B, C, D, E = roles(t)
        u = t + 1
        sched = 16 <= u < 80
        wt = f"w{t & 15}"
        wu = f"w{u & 15}"
        if sched:
            ins.append(("v_bitop3_b32", "t2", f"w{(u - 3) & 15}", f"w{(u - 8) & 15}", f"w{(u - 14) & 15}", 0x96))
        e_src = R.rd(E)
        ins.append(("v_add3_u32", R.wr(E), e_src, f"k{t // 20}", wt))
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        if sched:
            ins.append(("v_xor_b32", wu, "t2", wu))
        ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        if sched:
            ins.append(("v_alignbit_b32", wu, wu, wu, 31))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
    assert R.cur == [f"r{i}" for i in range(5)]
    return ins


def ring_reg(q: int, j: int) -> str:
    return f"v{RING_BASE + 4 * (q % RING_QUADS) + j}"


def gen_lds():
    """SHA1_LDS instruction list. Operands: r0-4 (out), t0-1 (tmp), h0-4 (in), addr (vgpr in),
    k0-3 (sgpr in).  Reads quad g (W[4g..4g+3]) from addr + g*1024."""
    ins = [("s_waitcnt_lgkm", 0)]
    ahead = RING_QUADS - 1
    issued = -1
    for g in range(min(ahead, 20)):
        ins.append(("ds_read_b128", g, g * 1024))
        issued = g
    R = Regs()
    for t in range(80):
        g = t // 4
        if t % 4 == 0:
            ins.append(("s_waitcnt_lgkm", issued - g))
        A, B, C, D, E = roles(t)
        e_src = R.rd(E)
        ins.append(("v_add3_u32", R.wr(E), e_src, f"k{t // 20}", ring_reg(g, t % 4)))
        if t % 4 == 3 and g + ahead < 20:
            ins.append(("ds_read_b128", g + ahead, (g + ahead) * 1024))
            issued = g + ahead
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
    assert R.cur == [f"r{i}" for i in range(5)]
    return ins


# ---------------------------------------------------------------- emulator -------------

def emulate(ins, regs: dict, lds: dict | None = None, addr: int = 0):
    """Execute an instruction list on a dict of 32-bit registers (one lane)."""

    def v(x):
        return regs[x] if isinstance(x, str) else x

    for op in ins:
        o = op[0]
        if o == "v_add3_u32":
            regs[op[1]] = (v(op[2]) + v(op[3]) + v(op[4])) & M32
        elif o == "v_alignbit_b32":
            s = op[4] & 31
            cat = (v(op[2]) << 32) | v(op[3])
            regs[op[1]] = (cat >> s) & M32
        elif o == "v_bfi_b32":
            a, b, c = v(op[2]), v(op[3]), v(op[4])
            regs[op[1]] = ((a & b) | (~a & c)) & M32
        elif o == "v_bitop3_b32":
            a, b, c, imm = v(op[2]), v(op[3]), v(op[4]), op[5]
            r = 0
            for bit in range(32):
                idx = (((a >> bit) & 1) << 2) | (((b >> bit) & 1) << 1) | ((c >> bit) & 1)
                r |= ((imm >> idx) & 1) << bit
            regs[op[1]] = r
        elif o == "v_xor_b32":
            regs[op[1]] = v(op[2]) ^ v(op[3])
        elif o == "ds_read_b128":
            q, off = op[1], op[2]
            for j in range(4):
                regs[ring_reg(q, j)] = lds[addr + off + 4 * j]
        elif o == "s_waitcnt_lgkm":
            pass
        else:
            raise ValueError(o)
    return regs


def _check_block(block: bytes, h):
    w = list(struct.unpack(">16I", block))
    # expected: reference compress
    def rotl(x, n):
        return ((x << n) | (x >> (32 - n))) & M32
    ww = w + [0] * 64
    for t in range(16, 80):
        ww[t] = rotl(ww[t - 3] ^ ww[t - 8] ^ ww[t - 14] ^ ww[t - 16], 1)
    a, b, c, d, e = h
    for t in range(80):
        if t < 20:
            f = (b & c) | (~b & d)
        elif t < 40 or t >= 60:
            f = b ^ c ^ d
        else:
            f = (b & c) | (b & d) | (c & d)
        tmp = (rotl(a, 5) + (f & M32) + e + K[t // 20] + ww[t]) & M32
        e, d, c, b, a = d, c, rotl(b, 30), a, tmp
    exp = [(x + y) & M32 for x, y in zip(h, (a, b, c, d, e))]

    base = {f"h{i}": h[i] for i in range(5)}
    base.update({f"k{i}": K[i] for i in range(4)})
    # FULL
    regs = dict(base)
    regs.update({f"w{i}": w[i] for i in range(16)})
    emulate(gen_full(), regs)
    got = [(h[i] + regs[f"r{i}"]) & M32 for i in range(5)]
    assert got == exp, "SHA1_FULL mismatch"
    # LDS
    regs = dict(base)
    lds = {}
    for t in range(80):
        lds[1024 * (t // 4) + 4 * (t % 4)] = ww[t]
    emulate(gen_lds(), regs, lds, 0)
    got = [(h[i] + regs[f"r{i}"]) & M32 for i in range(5)]
    assert got == exp, "SHA1_LDS mismatch"
    return exp


def self_check():
    """Hash several messages through the emulated instruction streams; compare with hashlib."""
    import random
    rng = random.Random(1)
    for n in [0, 3, 55, 56, 64, 119, 200]:
        msg = bytes(rng.randrange(256) for _ in range(n))
        bits = 8 * n
        padded = msg + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", bits)
        h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        for i in range(0, len(padded), 64):
            h = _check_block(padded[i:i + 64], h)
        assert struct.pack(">5I", *h) == hashlib.sha1(msg).digest(), n
    return True


# ---------------------------------------------------------------- emitter --------------

def _opnd(x, full: bool):
    if isinstance(x, int):
        return str(x)
    if x.startswith("v") and x[1:].isdigit():
        return x  # physical ring register
    return f"%[{x}]"


def emit(ins, full: bool) -> str:
    lines = []
    for op in ins:
        o = op[0]
        if o == "s_waitcnt_lgkm":
            lines.append(f"s_waitcnt lgkmcnt({op[1]})")
        elif o == "ds_read_b128":
            q, off = op[1], op[2]
            lo = RING_BASE + 4 * (q % RING_QUADS)
            lines.append(f"ds_read_b128 v[{lo}:{lo + 3}], %[addr] offset:{off}")
        elif o == "v_bitop3_b32":
            lines.append(f"v_bitop3_b32 {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}, "
                         f"{_opnd(op[4], full)} bitop3:0x{op[5]:02x}")
        elif o == "v_alignbit_b32":
            lines.append(f"v_alignbit_b32 {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}, {op[4]}")
        elif o == "v_xor_b32":
            lines.append(f"v_xor_b32 {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}")
        else:
            lines.append(f"{o} " + ", ".join(_opnd(x, full) for x in op[1:]))
    return "\n".join(f'    "{l}\\n"' for l in lines)


HEADER = """// GENERATED by tools/gen_sha1_asm.py -- do not edit.  Regenerate with:
//   python3 tools/gen_sha1_asm.py
// The instruction streams below are checked against hashlib by the generator's emulator
// (tests/test_asm_gen.py) before they are written.
#pragma once
#include <stdint.h>

#define TV_SHA1_RING_BASE {ring_base}
#define TV_SHA1_RING_QUADS {ring_quads}

// One SHA-1 compression, schedule in-asm.  w[16] holds the big-endian message words and is
// clobbered.  On return r = working state after round 79; caller does h += r.
__device__ __forceinline__ void tv_sha1_full(const uint32_t h[5], uint32_t r[5], uint32_t w[16],
                                             uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t t0, t1, t2;
    asm(
{full}
    : [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [w0] "+v"(w[0]), [w1] "+v"(w[1]), [w2] "+v"(w[2]), [w3] "+v"(w[3]),
      [w4] "+v"(w[4]), [w5] "+v"(w[5]), [w6] "+v"(w[6]), [w7] "+v"(w[7]),
      [w8] "+v"(w[8]), [w9] "+v"(w[9]), [w10] "+v"(w[10]), [w11] "+v"(w[11]),
      [w12] "+v"(w[12]), [w13] "+v"(w[13]), [w14] "+v"(w[14]), [w15] "+v"(w[15]),
      [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
    : [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]), [h4] "v"(h[4]),
      [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3));
}}

// The 80 rounds of one compression with W[0..79] read from LDS at byte address `addr`
// (+ g*1024 for quad g).  Waits for all of its own LDS reads before returning.
__device__ __forceinline__ void tv_sha1_lds(const uint32_t h[5], uint32_t r[5], uint32_t addr,
                                            uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t t0, t1;
    asm volatile(
{lds}
    : [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [t0] "=&v"(t0), [t1] "=&v"(t1)
    : [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]), [h4] "v"(h[4]),
      [addr] "v"(addr), [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {clobbers}, "memory");
}}
"""


def render() -> str:
    clob = ", ".join(f'"v{RING_BASE + i}"' for i in range(4 * RING_QUADS))
    return HEADER.format(ring_base=RING_BASE, ring_quads=RING_QUADS, full=emit(gen_full(), True),
                         lds=emit(gen_lds(), False), clobbers=clob)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "torrent_amd", "csrc", "sha1_asm.h"))
    ap.add_argument("--check", action="store_true", help="only run the emulator self-check")
    a = ap.parse_args()
    self_check()
    if a.check:
        print("emulator self-check: ok")
        return
    txt = render()
    with open(a.out, "w") as f:
        f.write(txt)
    full = gen_full()
    lds = gen_lds()
    print(f"wrote {a.out}: FULL {len(full)} instr, LDS {len(lds)} instr")


if __name__ == "__main__":
    sys.exit(main())
