#!/usr/bin/env python3
"""Generate torrent_amd/csrc/sha1_asm.h: gfx950 inline-asm SHA-1 compression blocks.

Why generated asm: hipcc (ROCm 7.2) does not fold XOR3 / Maj into v_bitop3_b32 (one
compression compiles to ~790 VALU instead of ~613), and it pads every inline-asm boundary
with `s_nop 0`, which costs a full issue slot for a lone wave.  So each compression is ONE
asm statement, and this script emits it.  The emitted instruction stream is executed by the
emulator below against hashlib before the header is written (`--check`, also run by
tests/test_abi.py::test_asm_generator_emulator), so a wrong register rotation can never reach the GPU.

Blocks emitted
--------------
SHA1_FULL   one 64-byte block, message schedule computed in-asm (16-word rolling window).
            5 VALU per round + 3 per scheduled word = 400 + 192 = 592 (+16 v_perm bswap and
            5 feed-forward adds by the compiler outside) = 613 per block.
SHA1_LDS    the 80 rounds only (400 VALU); W[0..79] comes from LDS as 20 ds_read_b128
            (layout [t/4][lane][4 words], conflict-free), kept 15 quads ahead in an 80-VGPR
            ring of PHYSICAL registers (a 128-bit asm operand cannot be split in AMDGPU asm).
            The split kernel's rounds loop is one pipelined stream over its blocks: the reads
            run 15 quads ahead across block boundaries (gen_rounds_block; 3 LDS buffers, the
            helper two blocks ahead), checked by check_rounds_stream against the helper's
            protocol.

Round (roles rotate statically; the new `a` is written into the old `e` register):
    E  = v_add3_u32(E, K, W[t])          # off the critical path
    T0 = v_alignbit_b32(A, A, 27)        # rotl5(a)
    T1 = f(B, C, D)                      # v_bitop3_b32 0xCA (Ch) / 0x96 (Parity) / 0xE8 (Maj)
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

# physical VGPRs used by SHA1_LDS for its K+W ring (quad-aligned; a 128-bit asm operand cannot
# be split in AMDGPU asm).  The kernel's VGPR count is therefore >= RING_BASE + 4*RING_QUADS.
# A ds_read_b128 of a wave64 returns 1 KiB and its latency under the rounds wave's VALU stream is
# long: 15 quads in flight (60 rounds ahead, lgkmcnt's 4-bit maximum) run the 80-round block in
# 1,794 cycles against 1,894 with 7 in flight (tools/gen_ubench_rounds.py, profiles/r01/ubench_rounds.log).
RING_BASE = 64
# (the TV_GEN_* environment variables select build variants for A/B measurements; the defaults are
# the shipped configuration)
RING_QUADS = int(os.environ.get("TV_GEN_RING", "16"))   # register quads of the K+W ring
READ_AHEAD = int(os.environ.get("TV_GEN_RA", "15"))   # quads in flight ahead of the one being consumed
WAIT_EVERY = int(os.environ.get("TV_GEN_WAIT", "4"))    # one s_waitcnt per WAIT_EVERY quads
LDS_BUFS = int(os.environ.get("TV_GEN_BUFS", "3"))      # K+W buffers per pair; the helper runs LDS_BUFS-1 blocks ahead
# PIPELINED = 1: the rounds reads run 15 quads ahead ACROSS block boundaries (gen_rounds_block).  Measured
# 4 % slower than a burst of 15 reads at each block's start (13.69 vs 12.95 ms at cfg2,
# profiles/r02/split_variants.jsonl): LDS data returning under the VALU stream costs more issue cycles
# than a burst landing while the wave waits.  Kept as a checked option; the shipped build is 0.
PIPELINED = os.environ.get("TV_GEN_PIPE", "0") == "1"
PAIR_XOR = os.environ.get("TV_GEN_PAIRXOR", "1") == "1"   # lane compression: schedule words two at a time
ALIGN_FULL = os.environ.get("TV_GEN_ALIGN", "1") == "1"   # lane compression block starts 8-byte aligned
HELPER_PAIR = os.environ.get("TV_GEN_HPAIR", "0") == "1"  # split helper: schedule in pairs (4-byte ops paired)
K_IN_ROUNDS = os.environ.get("TV_GEN_KROUNDS", "0") == "1"  # split: the rounds wave adds K (v_add3 with an SGPR)
HELPER_X = os.environ.get("TV_GEN_HX", "")   # timing probes only: novalu / nowrite / noload (digests are wrong)
ROUNDS_X = os.environ.get("TV_GEN_RX", "")   # timing probe only: nowait = the split rounds loop without its LDS-return
                                             # waits (digests are wrong; barriers unchanged)
# Diagnostic builds only (tools/split_stamps.py): STAMP = 1 brackets the split kernel's in-loop barriers (rounds and
# helper waves) with shader-clock reads into SGPRs s[88:91] and accumulates the cycles spent at them in an SGPR
# operand; the kernels then need -DTV_STAMPS=1.  The default header is unchanged.
# STAMP = 2 also brackets the helper's two waits per block: for its prefetched global words (vmcnt) and for its
# LDS writes before the barrier (lgkmcnt), into %[svm] and %[slg].
STAMP = int(os.environ.get("TV_GEN_STAMP", "0"))


def _stamped(line: str, acc: str) -> list:
    return ["s_memtime s[88:89]", line, "s_memtime s[90:91]", "s_waitcnt lgkmcnt(0)",
            "s_sub_u32 s90, s90, s88", f"s_add_u32 %[{acc}], %[{acc}], s90"]


STAMP_SEQ = _stamped("s_barrier", "sbar")
# Split helper: where it waits for its LDS writes.  "0": lgkmcnt(0) before every barrier (block m's writes done
# before barrier m - 1).  "mid": lgkmcnt(10) before the 11th write of block m + 1 instead -- block m is read
# only after barrier m, and the next block's first 10 writes (issued after block m's, LDS counts in order) may
# still be in flight; nothing waits at the barrier.
HELPER_WAIT = os.environ.get("TV_GEN_HWAIT", "mid")
LOOP_ALIGN = os.environ.get("TV_GEN_LALIGN", "1") == "1"  # split loops: .p2align 3 before every block body
HELPER_AHEAD = LDS_BUFS - 1
assert not PIPELINED or (LDS_BUFS >= 3 and RING_QUADS == 20), "the pipelined stream needs 3 buffers and a 20-quad ring"
# physical VGPRs of the helper (schedule) block: 16-word W window, xor3 temp, 3 output quads
HW_BASE = 80
HT = 96
HT2 = 97   # second schedule temp (HELPER_PAIR)
HOUT_BASE = 100
HOUT_QUADS = 3


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
    # Ch as v_bitop3 0xCA, not v_bfi_b32: same 8-byte issue cost, but v_bitop3 runs at full rate on
    # the SIMD (2 cyc per wave64) and v_bfi at half rate (4 cyc; tools/ubench_simd.hip)
    return ("v_bitop3_b32", dst, b, c, d, {"ch": 0xCA, "par": 0x96}.get(k, 0xE8))


def gen_full():
    """SHA1_FULL instruction list. Operands: r0-4 (out), w0-15 (in/out), t0-3 (tmp),
    h0-4 (in), k0-3 (sgpr in).

    With PAIR_XOR the schedule words are computed two at a time (W[u], W[u+1] for even u, in round u-1)
    so that the two 4-byte v_xor_b32 of a pair sit next to each other: every other instruction of the
    block is an 8-byte VOP3, and an odd number of 4-byte instructions between them would leave every
    following VOP3 at an address = 4 mod 8.  A lone wave issues long runs of such misaligned 8-byte
    instructions at ~5.07 instead of 4.07 cycles (tools/ubench_align, profiles/r02/ubench_align.log); the
    block starts 8-byte aligned (".p2align 3" in the emitted text, ALIGN_FULL)."""
    ins = []
    R = Regs()
    for t in range(80):
        A, B, C, D, E = roles(t)
        wt = f"w{t & 15}"
        if PAIR_XOR:
            us = [t + 1, t + 2] if t % 2 == 1 and 15 <= t <= 77 else []   # pairs (16,17) .. (78,79)
            tmps = ["t2", "t3"]
            for i, u in enumerate(us):
                ins.append(("v_bitop3_b32", tmps[i], f"w{(u - 3) & 15}", f"w{(u - 8) & 15}", f"w{(u - 14) & 15}", 0x96))
            e_src = R.rd(E)
            ins.append(("v_add3_u32", R.wr(E), e_src, f"k{t // 20}", wt))
            ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
            for i, u in enumerate(us):
                ins.append(("v_xor_b32", f"w{u & 15}", tmps[i], f"w{u & 15}"))
            ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
            b_src = R.rd(B)
            ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
            for u in us:
                ins.append(("v_alignbit_b32", f"w{u & 15}", f"w{u & 15}", f"w{u & 15}", 31))
            ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
            continue
        u = t + 1
        sched = 16 <= u < 80
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


def gen_lds(off_base: int = 0, lead_wait: bool = True):
    """SHA1_LDS instruction list. Operands: r0-4 (out), t0-1 (tmp), h0-4 (in), addr (vgpr in).
    Quad g (K+W[4g..4g+3], K pre-added by the helper) is read from addr + off_base + g*1024."""
    ins = [("s_waitcnt_lgkm", 0)] if lead_wait else []
    issued = -1
    for g in range(min(READ_AHEAD, 20)):
        ins.append(("ds_read_b128", g, off_base + g * 1024))
        issued = g
    R = Regs()
    for t in range(80):
        g = t // 4
        if t % 4 == 0 and g % WAIT_EVERY == 0:
            need = min(g + WAIT_EVERY - 1, 19)          # quads consumed before the next wait
            ins.append(("s_waitcnt_lgkm", min(15, max(0, issued - need))))   # (lgkmcnt is 4 bits)
        A, B, C, D, E = roles(t)
        e_src = R.rd(E)
        if K_IN_ROUNDS:
            ins.append(("v_add3_u32", R.wr(E), e_src, f"k{t // 20}", ring_reg(g, t % 4)))
        else:
            ins.append(("v_add_u32", R.wr(E), ring_reg(g, t % 4), e_src))
        if t % 4 == 3 and g + READ_AHEAD < 20:
            ins.append(("ds_read_b128", g + READ_AHEAD, off_base + (g + READ_AHEAD) * 1024))
            issued = g + READ_AHEAD
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
    assert R.cur == [f"r{i}" for i in range(5)]
    return ins


def gen_rounds_block(off_cur: int, off_next: int):
    """One block of the split kernel's PIPELINED rounds stream.  On entry quads 0..14 of this block are in
    flight (issued by the previous block, or the loop prologue); after consuming quad g the read of quad
    g + 15 is issued -- past quad 19 that is quad g - 5 of the NEXT block, from its buffer at off_next -- so
    READ_AHEAD quads stay in flight across block boundaries and no block starts on an LDS latency bubble.
    Then h += r and the workgroup barrier.  Needs the helper two blocks ahead (LDS_BUFS = 3): the next
    block was written before the barrier that started this one."""
    ins = []
    R = Regs()
    allowed = READ_AHEAD - WAIT_EVERY   # reads still in flight once quads g .. g+WAIT_EVERY-1 retired
    for t in range(80):
        g = t // 4
        if t % 4 == 0 and g % WAIT_EVERY == 0:
            ins.append(("s_waitcnt_lgkm", allowed))
        A, B, C, D, E = roles(t)
        e_src = R.rd(E)
        if K_IN_ROUNDS:
            ins.append(("v_add3_u32", R.wr(E), e_src, f"k{t // 20}", ring_reg(g, t % 4)))
        else:
            ins.append(("v_add_u32", R.wr(E), ring_reg(g, t % 4), e_src))
        if t % 4 == 3:
            q = g + READ_AHEAD
            ins.append(("ds_read_b128", q % 20, off_cur + q * 1024 if q < 20 else off_next + (q - 20) * 1024))
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
    assert R.cur == [f"r{i}" for i in range(5)]
    for i in range(5):
        ins.append(("v_add_u32", f"h{i}", f"h{i}", f"r{i}"))
    ins.append(("s_barrier",))
    return ins


SPLIT_MID = os.environ.get("TV_GEN_SPLIT_MID", "0") == "1"   # split rounds loop: next block's reads mid-block
SPLIT_PRE = os.environ.get("TV_GEN_SPLIT_PRE", "0") == "1"   # split rounds loop: next block's 15 reads after round 79


def gen_split_pre_block(off_cur: int, off_next: int):
    """One block of the split rounds wave whose first READ_AHEAD reads were issued by the previous block: the
    shipped per-block stream (gen_lds) without its leading reads, followed after round 79 by the next block's
    leading reads (so they land during h += r and the barrier instead of after it), then h += r and the
    barrier.  Safe for the same reason as the twin kernel's: the next block was written before the barrier
    that started this one, and its buffer is not rewritten before the barrier that ends it."""
    body = gen_lds(off_cur, lead_wait=False)
    lead = [op for op in body[:READ_AHEAD] if op[0] == "ds_read_b128"]
    assert len(lead) == READ_AHEAD
    ins = body[READ_AHEAD:]
    ins += [("ds_read_b128", q, off_next + q * 1024) for q in range(READ_AHEAD)]
    for i in range(5):
        ins.append(("v_add_u32", f"h{i}", f"h{i}", f"r{i}"))
    ins.append(("s_barrier",))
    return ins


def gen_split_mid_block(off_cur: int, off_next: int):
    """One block of the split rounds wave with the NEXT block's first 10 K+W quads issued inside this block (the
    twin kernel's mid-block issue, tools/gen_sha1_asm.py gen_twin): on entry quads 0-9 of this block are in
    flight; it issues quads 10-14 at its start, quad 15+g after consuming quad g (g < 5), the next block's quads
    0-4 after round 39 and 5-9 after round 59 (each batch behind a wait that keeps at most 15 reads in flight,
    lgkmcnt's 4-bit limit), then h += r and the barrier.  Ring of 20 register quads, slot = quad.  The helper's
    protocol makes it safe: the next block was written before the barrier that started this one."""
    assert RING_QUADS == 20
    ins, order = [], [("cur", q) for q in range(10)]   # reads in flight on entry, oldest first
    retired = 0                                         # reads of `order` known retired

    def wait_for(key):
        nonlocal retired
        i = order.index(key)
        if i >= retired:
            ins.append(("s_waitcnt_lgkm", min(15, len(order) - 1 - i)))
            retired = i + 1

    def issue(tag, q):
        assert len(order) - retired < 15 or True
        ins.append(("ds_read_b128", q, (off_cur if tag == "cur" else off_next) + q * 1024))
        order.append((tag, q))

    for q in range(10, 15):
        issue("cur", q)
    R = Regs()
    for t in range(80):
        g = t // 4
        if t % 4 == 0:
            wait_for(("cur", g))
        A, B, C, D, E = roles(t)
        e_src = R.rd(E)
        ins.append(("v_add_u32", R.wr(E), ring_reg(g, t % 4), e_src))
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
        if t % 4 == 3 and g < 5:
            issue("cur", 15 + g)
        if t == 39:
            wait_for(("cur", 14))
            for q in range(5):
                issue("next", q)
        if t == 59:
            wait_for(("cur", 19))
            for q in range(5, 10):
                issue("next", q)
    assert R.cur == [f"r{i}" for i in range(5)]
    # at most 15 in flight at every issue, counting every read not yet waited for as in flight
    inflight, waited = 0, 0
    for op in ins:
        if op[0] == "ds_read_b128":
            inflight += 1
            assert inflight <= 15, "more than 15 LDS reads in flight"
        elif op[0] == "s_waitcnt_lgkm":
            inflight = min(inflight, op[1])
    for i in range(5):
        ins.append(("v_add_u32", f"h{i}", f"h{i}", f"r{i}"))
    ins.append(("s_barrier",))
    return ins


def rounds_prologue(off: int = 0):
    """Issue quads 0 .. READ_AHEAD-1 of the first block (buffer at off)."""
    return [("ds_read_b128", g, off + g * 1024) for g in range(READ_AHEAD)]


def hw(t: int) -> str:
    return f"v{HW_BASE + (t & 15)}"


def gen_helper(src=None, off_base: int = 0):
    """Helper (schedule) block: src = 16 registers holding the block's words as loaded
    (little-endian; default operands raw0-15), sel (sgpr 0x00010203), addr (vgpr, LDS byte address
    of this lane in ring buffer 0), k0-3 (sgpr).  Writes K+W[t] for t = 0..79 to LDS at
    addr + off_base + (t/4)*1024 as [t/4][lane][4] (one ds_write_b128 per quad).
    With HELPER_PAIR the schedule of a quad runs as two pairs (W[t], W[t+1]), each bitop3, bitop3, xor,
    xor, alignbit, alignbit, so the 4-byte instructions (the xors and the four K adds) come in pairs and
    the 8-byte ones keep their alignment."""
    if src is None:
        src = [f"raw{i}" for i in range(16)]
    ins = []
    for i in range(16):
        ins.append(("v_perm_b32", hw(i), 0, src[i], "sel"))
    for q in range(20):
        if q >= 4 and HELPER_PAIR:
            for p in range(2):
                ts = (4 * q + 2 * p, 4 * q + 2 * p + 1)
                tmp = (f"v{HT}", f"v{HT2}")
                for i, t in enumerate(ts):
                    ins.append(("v_bitop3_b32", tmp[i], hw(t - 3), hw(t - 8), hw(t - 14), 0x96))
                for i, t in enumerate(ts):
                    ins.append(("v_xor_b32", hw(t), tmp[i], hw(t)))
                for t in ts:
                    ins.append(("v_alignbit_b32", hw(t), hw(t), hw(t), 31))
        elif q >= 4:
            for i in range(4):
                t = 4 * q + i
                ins.append(("v_bitop3_b32", f"v{HT}", hw(t - 3), hw(t - 8), hw(t - 14), 0x96))
                ins.append(("v_xor_b32", hw(t), f"v{HT}", hw(t)))
                ins.append(("v_alignbit_b32", hw(t), hw(t), hw(t), 31))
        qoff = off_base + q * 1024
        if K_IN_ROUNDS:     # the rounds wave adds K: W[4q..4q+3] go to LDS straight from the window
            ins.append(("ds_write_b128", HW_BASE + ((4 * q) & 15), qoff))
            continue
        o = HOUT_BASE + 4 * (q % HOUT_QUADS)
        for j in range(4):
            ins.append(("v_add_u32", f"v{o + j}", f"k{q // 5}", hw(4 * q + j)))
        ins.append(("ds_write_b128", o, qoff))
    return ins


# ---- TWIN: two lanes per piece, in the rounds waves AND the helper waves ----
# A twin workgroup is 2 rounds waves + 2 helper waves over 64 pieces; in every wave lane 2i+b runs piece
# 32w+i and owns the schedule words of PARITY b.  Rounds: both lanes of a pair run the same 80 rounds on the
# same state; lane b reads only its own K+W words (10 ds_read_b128 per block instead of 20) and round t's
# `e + KW` add takes KW from lane t%2 of the pair through DPP (quad_perm [b,b,2+b,2+b]).  Helper: both lanes
# expand W[16..31] with the standard recurrence, then keep their own parity (v_perm with a per-lane selector)
# and expand W[32..79] with W[t] = rotl2(W[t-6] ^ W[t-16] ^ W[t-28] ^ W[t-32]), whose terms all have t's
# parity: 192 VALU + 10 ds_write_b128 per block and lane instead of 308 + 20 (gen_helper2).  Every round is
# five 8-byte instructions, so each 4-byte s_waitcnt is followed by `s_nop 0` to keep the stream 8-byte
# aligned (a long misaligned run issues at ~5.07 instead of 4.07 cycles), with two waits per block: before
# round 0 (reads 0-4) and round 40 (reads 5-9).  Buffer layout [k][wave][lane][4 words]: lane 2i+b of wave w
# holds W[8k+b], W[8k+b+2], W[8k+b+4], W[8k+b+6] (+K) of piece 32w+i at k*2048 + w*1024 + lane*16, written
# and read as one contiguous KiB per wave (tools/gen_ubench_dpp.py, profiles/r02/ubench_dpp.log: the rounds
# stream alone 1,723-1,758 vs 1,818 cycles per block for the shipped 20-read stream).
TWIN_READ_BYTES = 2048
TWIN_WAITS = tuple(int(x) for x in os.environ.get("TV_GEN_TWIN_WAITS", "0-5").split("-"))   # reads waited for, in pairs
TWIN_PRE = os.environ.get("TV_GEN_TWIN_PRE", "1") == "1"   # loop: issue the next block's reads after round 79
TWIN_NONOP = os.environ.get("TV_GEN_TWIN_NONOP", "1") == "1"  # loop: 4-byte instructions paired without s_nop
# 64-byte placement of the twin loops: rounds loop head at (4 + 8 k) mod 64 for TV_GEN_TWIN_RALIGN = k, helper
# loop head at 4 m mod 64 for TV_GEN_TWIN_HALIGN = m ("none": wherever the code before them puts them).  The
# rounds loop at 4 mod 64 (and the helper's at 60) is 0.7-1.6 % faster at cfg2 than at 28, 52 or 60
# (profiles/r03/twin_ralign.jsonl: 11.89-11.91 vs 11.98-12.08 ms), so both are pinned there: a code change
# before the loops no longer moves them.
TWIN_RALIGN = os.environ.get("TV_GEN_TWIN_RALIGN", "0")
TWIN_HALIGN = os.environ.get("TV_GEN_TWIN_HALIGN", "15")
TWIN_RALIGN = None if TWIN_RALIGN == "none" else TWIN_RALIGN
TWIN_HALIGN = None if TWIN_HALIGN == "none" else TWIN_HALIGN
# the same for the split kernel's loops: rounds loop head at 8 k mod 64 (TV_GEN_SPLIT_RALIGN = k; its block
# bodies start with .p2align 3), helper loop head at 4 m mod 64 (TV_GEN_SPLIT_HALIGN = m).  At 25,600 pieces
# the rounds loop's eight placements are within 0.5 % of each other (profiles/r03/split_ralign.jsonl); k = 6
# (48 mod 64) was the fastest of the two rounds by 0.2 % and is pinned so that code changes cannot move it.
SPLIT_RALIGN = os.environ.get("TV_GEN_SPLIT_RALIGN", "6")
SPLIT_HALIGN = os.environ.get("TV_GEN_SPLIT_HALIGN")
SPLIT_RALIGN = None if SPLIT_RALIGN == "none" else SPLIT_RALIGN
# loop: when the next block's reads are issued -- "end": all 10 after round 79; "mid": 0-4 after the round-40
# wait, 5-9 after round 79; "spread": read k after round 8k+7 (each as soon as its registers are consumed)
TWIN_ISSUE = os.environ.get("TV_GEN_TWIN_ISSUE", "mid")   # mid: +1.8 % at cfg2 over end, spread -2 % (profiles/r02/twin_ab.jsonl.log)


def gen_twin(off_base: int = 0, reads_next: int | None = None, lead: bool = False):
    """TWIN rounds block.  lead: issue this block's own 10 reads first (tv_sha1_twin_lds); reads_next:
    after round 79 issue the 10 reads of the block whose buffer is at that offset (the loop body).
    Operands as gen_lds: r0-4 (out), t0-1 (tmp), h0-4 (in), addr (this lane's LDS byte address)."""
    ins = [("ds_read_b128", k, off_base + k * TWIN_READ_BYTES) for k in range(10)] if lead else []
    issue = TWIN_ISSUE if reads_next is not None else "end"
    assert issue == "end" or TWIN_WAITS == (0, 5)
    R = Regs()
    for t in range(80):
        k, b = t // 8, t % 2
        if issue == "spread" and t % 8 == 0 and t > 0:
            ins.append(("ds_read_b128", k - 1, reads_next + (k - 1) * TWIN_READ_BYTES))
        if t % 8 == 0 and k in TWIN_WAITS:
            nxt = [x for x in TWIN_WAITS if x > k]
            # reads k .. (next wait - 1) retired; "spread" has the next block's first 5 behind them at round 40
            ins.append(("s_waitcnt_lgkm", 5 if issue == "spread" and k == 5 else (10 - nxt[0] if nxt else 0)))
            ins.append(("s_nop",))
            if issue == "mid" and k == 5:
                ins += [("ds_read_b128", q, reads_next + q * TWIN_READ_BYTES) for q in range(5)]
        A, B, C, D, E = roles(t)
        e_src = R.rd(E)
        ins.append(("v_add_u32_dpp", R.wr(E), ring_reg(k, (t % 8) // 2), e_src, b))
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        ins.append(_fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
    assert R.cur == [f"r{i}" for i in range(5)]
    if reads_next is not None:
        first = {"end": 0, "mid": 5, "spread": 9}[issue]
        ins += [("ds_read_b128", k, reads_next + k * TWIN_READ_BYTES) for k in range(first, 10)]
    return ins


def rounds_loop_text() -> str:
    """The split kernel's rounds wave over nsteps (>= 1) blocks in which every lane updates, starting
    at ring buffer 0: one pipelined stream (gen_rounds_block) over buffers 0, 1, 2, 0, ... -- 80 rounds
    from K+W in LDS, h += r, barrier per block.  One asm statement, so no compiler bookkeeping or
    asm-boundary s_nop between blocks.  The reads issued ahead for the block after the last one are
    drained before it returns."""
    L = ["s_waitcnt lgkmcnt(0)", "s_mov_b32 %[cnt], %[nsteps]"]
    if PIPELINED:
        L.extend(_emit_lines(rounds_prologue(0)))
    if SPLIT_MID:
        L.extend(_emit_lines([("ds_read_b128", q, q * 1024) for q in range(10)]))
    if SPLIT_PRE:
        L.extend(_emit_lines([("ds_read_b128", q, q * 1024) for q in range(READ_AHEAD)]))
    if SPLIT_RALIGN is not None:
        L.append(".p2align 6")
        L.extend(["s_nop 0"] * (2 * int(SPLIT_RALIGN)))
    L.append("L_rloop_%=:")
    for k in range(LDS_BUFS):
        if SPLIT_PRE:
            if LOOP_ALIGN:
                L.append(".p2align 3")
            L.extend(_emit_lines(gen_split_pre_block(k * RING_BYTES, ((k + 1) % LDS_BUFS) * RING_BYTES)))
        elif SPLIT_MID:
            if LOOP_ALIGN:
                L.append(".p2align 3")
            L.extend(_emit_lines(gen_split_mid_block(k * RING_BYTES, ((k + 1) % LDS_BUFS) * RING_BYTES)))
        elif PIPELINED:
            L.extend(_emit_lines(gen_rounds_block(k * RING_BYTES, ((k + 1) % LDS_BUFS) * RING_BYTES)))
        else:   # per-block stream: its 15 reads issued at the block's start
            if LOOP_ALIGN:
                L.append(".p2align 3")
            body = _emit_lines(gen_lds(k * RING_BYTES, lead_wait=False))
            if ROUNDS_X == "nowait":
                body = [x for x in body if not x.startswith("s_waitcnt")]
            L.extend(body)
            L.extend(f"v_add_u32 %[h{i}], %[h{i}], %[r{i}]" for i in range(5))
            L.extend(STAMP_SEQ if STAMP else ["s_barrier"])   # (every LDS read of the block has been waited)
        L += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0",
              "s_cbranch_scc1 L_rdone_%=" if k < LDS_BUFS - 1 else "s_cbranch_scc0 L_rloop_%="]
    L += ["L_rdone_%=:", "s_waitcnt lgkmcnt(0)"]
    return "\n".join(f'    "{l}\\n"' for l in L)


H2_F, H2_P, H2_T, H2_O = 160, 192, 232, 236   # helper2 physical VGPRs: W[0..31], own-parity P[0..39], tmp, 3 out quads


def gen_helper2(src=None, off_base: int = 0):
    """TWIN helper block for a lane pair: src = the 16 registers holding the block's words as loaded
    (little-endian; default raw0-15, identical in both lanes), sel (sgpr 0x00010203), psel (vgpr: 0x03020100 in
    lane 0, 0x07060504 in lane 1 of each pair), addr (vgpr, this lane's LDS byte address), k0-3 (sgpr).  Lane b
    writes K+W[8k+b+2i] (i = 0..3) to addr + off_base + k*2048 for k = 0..9."""
    if src is None:
        src = [f"raw{i}" for i in range(16)]
    F = lambda t: f"v{H2_F + t}"      # noqa: E731  W[t], t < 32 (both parities)
    P = lambda j: f"v{H2_P + j}"      # noqa: E731  W[2j + b]
    T = f"v{H2_T}"
    ins = []
    nq = [0]

    def quad(k):   # K+W of own-parity words 4k..4k+3 -> LDS
        o = H2_O + 4 * (nq[0] % 3)
        nq[0] += 1
        for i in range(4):
            ins.append(("v_add_u32", f"v{o + i}", f"k{(4 * k + i) // 10}", P(4 * k + i)))
        ins.append(("ds_write_b128", o, off_base + k * TWIN_READ_BYTES))

    for i in range(16):
        ins.append(("v_perm_b32", F(i), 0, src[i], "sel"))
    for t in range(16, 32):
        ins.append(("v_bitop3_b32", T, F(t - 3), F(t - 8), F(t - 14), 0x96))
        ins.append(("v_xor_b32", F(t), T, F(t - 16)))
        ins.append(("v_alignbit_b32", F(t), F(t), F(t), 31))
    for j in range(16):
        ins.append(("v_perm_b32", P(j), F(2 * j + 1), F(2 * j), "psel"))
        if j % 4 == 3:
            quad(j // 4)
    for j in range(16, 40):
        ins.append(("v_bitop3_b32", T, P(j - 3), P(j - 8), P(j - 14), 0x96))
        ins.append(("v_xor_b32", P(j), T, P(j - 16)))
        ins.append(("v_alignbit_b32", P(j), P(j), P(j), 30))
        if j % 4 == 3:
            quad(j // 4)
    return ins


def twin_rounds_loop_text() -> str:
    """The TWIN rounds wave over nsteps (>= 1) blocks starting at ring buffer 0: the first block's reads,
    then per block gen_twin (its last instructions issue the next block's reads), h += r, barrier.  The
    reads issued after the final block (of the helper's spare block) are drained before it returns.
    Safe because the helper runs two blocks ahead: block j + 1 was written before the barrier that
    started block j, and buffer (j + 1) % 3 is not rewritten until after the barrier that ends block j + 1."""
    L = ["s_waitcnt lgkmcnt(0)", "s_mov_b32 %[cnt], %[nsteps]"]
    if TWIN_PRE:
        L.extend(_emit_lines([("ds_read_b128", k, k * TWIN_READ_BYTES) for k in range(10)]))
    if TWIN_PRE and TWIN_WAITS == (0, 5) and TWIN_NONOP:
        # No s_nop inside the loop: a block's 4-byte instructions come in even groups between its 8-byte runs.
        # The first wait sits at 4 mod 8 (the previous block's tail -- four 4-byte h adds, barrier, s_cmp,
        # s_cbranch -- precedes it; h0 += r0 is the 8-byte VOP3 form), and the loop counter's s_sub pairs
        # with the round-40 wait.
        if TWIN_RALIGN is not None:
            L += [".p2align 6"] + ["s_nop 0"] * (1 + 2 * int(TWIN_RALIGN)) + ["L_rloop_%=:"]
        else:
            L += [".p2align 3", "s_nop 0", "L_rloop_%=:"]
        for k in range(LDS_BUFS):
            body = _emit_lines(gen_twin(k * RING_BYTES, reads_next=((k + 1) % LDS_BUFS) * RING_BYTES))
            nops = [i for i, x in enumerate(body) if x == "s_nop 0"]
            assert len(nops) == 2 and body[nops[0] - 1].startswith("s_waitcnt") and nops[0] == 1
            body[nops[1]] = "s_sub_u32 %[cnt], %[cnt], 1"
            del body[nops[0]]
            L.extend(body)
            L.append("v_add_u32_e64 %[h0], %[h0], %[r0]")
            L.extend(f"v_add_u32 %[h{i}], %[h{i}], %[r{i}]" for i in range(1, 5))
            L += (STAMP_SEQ if STAMP else ["s_barrier"]) + ["s_cmp_eq_u32 %[cnt], 0",
                  "s_cbranch_scc1 L_rdone_%=" if k < LDS_BUFS - 1 else "s_cbranch_scc0 L_rloop_%="]
        L += ["L_rdone_%=:", "s_waitcnt lgkmcnt(0)"]
        return "\n".join(f'    "{l}\\n"' for l in L)
    L.append("L_rloop_%=:")
    for k in range(LDS_BUFS):
        L.append(".p2align 3")
        if TWIN_PRE:
            L.extend(_emit_lines(gen_twin(k * RING_BYTES, reads_next=((k + 1) % LDS_BUFS) * RING_BYTES)))
        else:
            L.extend(_emit_lines(gen_twin(k * RING_BYTES, lead=True)))
        L.extend(f"v_add_u32 %[h{i}], %[h{i}], %[r{i}]" for i in range(5))
        L.append("s_barrier")
        L += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0",
              "s_cbranch_scc1 L_rdone_%=" if k < LDS_BUFS - 1 else "s_cbranch_scc0 L_rloop_%="]
    L += ["L_rdone_%=:", "s_waitcnt lgkmcnt(0)"]
    return "\n".join(f'    "{l}\\n"' for l in L)


P0_BASE, P1_BASE, VL = 112, 128, 144   # prefetch buffers (2 blocks) and the running load pointer
RING_BYTES = 80 * 64 * 4               # one K+W buffer (also used by rounds_loop_text)


def helper_loop_text(twin: bool = False) -> str:
    """The helper wave's steady state as ONE asm statement (text, not emulated: its body is
    gen_helper, which the emulator checks).  For each raw block: wait for its prefetched words,
    byte-swap them, issue the loads 2 blocks ahead into the freed registers, expand the schedule,
    write K+W to LDS, barrier.  Loads land in physical registers the compiler never sees, so no
    compiler copy can touch an in-flight register and no compiler wait drains the prefetch."""
    L = []

    def loads(base):
        for q in range(4):
            L.append(f"global_load_dwordx4 v[{base + 4 * q}:{base + 4 * q + 3}], v[{VL}:{VL + 1}], off offset:{16 * q}")

    def advance():
        L.append("s_cmp_gt_u32 %[adv], 0")
        L.append("s_cselect_b64 %[inc], 64, 0")
        L.append("s_subb_u32 %[adv], %[adv], 0")
        L.append(f"v_lshl_add_u64 v[{VL}:{VL + 1}], v[{VL}:{VL + 1}], 0, %[inc]")

    def step(pbase, off_base, barrier=True):
        L.extend(_stamped("s_waitcnt vmcnt(4)", "svm") if STAMP >= 2 else ["s_waitcnt vmcnt(4)"])
        body = (gen_helper2 if twin else gen_helper)([f"v{pbase + i}" for i in range(16)], off_base)
        perms, rest = body[:16], body[16:]
        # timing-only experiments (wrong digests): drop a class of the helper's work, keep its barriers
        if HELPER_X == "novalu":
            rest = [op for op in rest if op[0] == "ds_write_b128"]
        elif HELPER_X == "nowrite":
            rest = [op for op in rest if op[0] != "ds_write_b128"]
        if LOOP_ALIGN:
            L.append(".p2align 3")
        L.extend(_emit_lines(perms))
        if HELPER_X != "noload":
            loads(pbase)    # the perms have read pbase: refill it with the block 2 ahead
        advance()
        if LOOP_ALIGN:
            L.append(".p2align 3")
        if HELPER_WAIT == "mid" and not twin:
            assert HELPER_AHEAD >= 2
            k = [i for i, op in enumerate(rest) if op[0] == "ds_write_b128"][10]
            rest = rest[:k] + [("s_waitcnt_lgkm", 10)] + rest[k:]
        L.extend(_emit_lines(rest))
        if barrier and HELPER_WAIT == "mid" and not twin:
            L.extend(STAMP_SEQ if STAMP else ["s_barrier"])
        elif barrier:
            L.extend(_stamped("s_waitcnt lgkmcnt(0)", "slg") if STAMP >= 2 else ["s_waitcnt lgkmcnt(0)"])
            L.extend(STAMP_SEQ if STAMP else ["s_barrier"])

    L.append("s_sub_u32 %[adv], %[nraw], 1")
    L.append(f"v_mov_b64 v[{VL}:{VL + 1}], %[va]")
    loads(P0_BASE)
    advance()
    loads(P1_BASE)
    advance()
    # block 0 into buffer 0; with the helper A = HELPER_AHEAD blocks ahead no barrier follows its first A - 1
    # writes: its first barrier (the rounds wave's starting one) follows the write of block A - 1, and block m
    # (m >= A - 1) is followed by barrier m - A + 2 -- the C++ tail's rule (b - b0 + 1 >= kAhead) -- so the
    # helper, whose A - 1 extra barriers end it, executes as many barriers as the rounds wave
    step(P0_BASE, 0, barrier=HELPER_AHEAD == 1)
    L.append("s_sub_u32 %[cnt], %[nraw], 1")
    L.append("s_cmp_eq_u32 %[cnt], 0")
    L.append("s_cbranch_scc1 L_hdone_%=")
    first_loop_blk = max(1, HELPER_AHEAD - 1)
    for m in range(1, first_loop_blk):   # blocks 1 .. A - 2 (A >= 3): written before the first barrier
        step((P0_BASE, P1_BASE)[m % 2], (m % LDS_BUFS) * RING_BYTES, barrier=False)
        L.append("s_sub_u32 %[cnt], %[cnt], 1")
        L.append("s_cmp_eq_u32 %[cnt], 0")
        L.append("s_cbranch_scc1 L_hdone_%=")
    if twin and TWIN_HALIGN is not None:
        L.append(".p2align 6")
        L.extend(["s_nop 0"] * int(TWIN_HALIGN))
    if not twin and SPLIT_HALIGN is not None:
        L.append(".p2align 6")
        L.extend(["s_nop 0"] * int(SPLIT_HALIGN))
    L.append("L_hloop_%=:")
    period = 2 * LDS_BUFS // (2 if LDS_BUFS % 2 == 0 else 1)   # lcm(prefetch register sets 2, LDS buffers)
    for k in range(period):
        blk = k + first_loop_blk     # block index (mod period) of this step
        step((P0_BASE, P1_BASE)[blk % 2], (blk % LDS_BUFS) * RING_BYTES)
        L.append("s_sub_u32 %[cnt], %[cnt], 1")
        L.append("s_cmp_eq_u32 %[cnt], 0")
        L.append("s_cbranch_scc1 L_hdone_%=" if k < period - 1 else "s_cbranch_scc0 L_hloop_%=")
    L.append("L_hdone_%=:")
    if HELPER_WAIT == "mid" and not twin:
        L.append("s_waitcnt lgkmcnt(0)")   # (no write of this statement left in flight for the compiler's code)
    L.append("s_waitcnt vmcnt(0)")
    return "\n".join(f'    "{l}\\n"' for l in L)


# ---------------------------------------------------------------- emulator -------------

def emulate(ins, regs: dict, lds: dict | None = None, addr: int = 0, on_barrier=None, drain: bool = True,
            pending: list | None = None):
    """Execute an instruction list on a dict of 32-bit registers (one lane).  ds_read results
    land only when an s_waitcnt lgkmcnt(N) retires them (in order); reading a register whose
    load is still in flight, or overwriting one, raises -- so the wait counts are checked too.
    `pending` (the lane's in-flight reads) may be passed in to carry it across calls."""
    if pending is None:
        pending = []  # [(regs, values, lds addresses)] oldest first

    def v(x):
        if isinstance(x, str):
            for rs, _, _ in pending:
                if x in rs:
                    raise AssertionError(f"read of {x} before its ds_read retired")
            return regs[x]
        return x

    def wr(x, val):
        for rs, _, _ in pending:
            if x in rs:
                raise AssertionError(f"write of {x} while its ds_read is in flight")
        regs[x] = val

    for op in ins:
        o = op[0]
        if o == "v_add3_u32":
            wr(op[1], (v(op[2]) + v(op[3]) + v(op[4])) & M32)
        elif o == "v_alignbit_b32":
            s_ = op[4] & 31
            cat = (v(op[2]) << 32) | v(op[3])
            wr(op[1], (cat >> s_) & M32)
        elif o == "v_bfi_b32":
            a, b, c = v(op[2]), v(op[3]), v(op[4])
            wr(op[1], ((a & b) | (~a & c)) & M32)
        elif o == "v_bitop3_b32":
            a, b, c, imm = v(op[2]), v(op[3]), v(op[4]), op[5]
            r = 0
            for bit in range(32):
                idx = (((a >> bit) & 1) << 2) | (((b >> bit) & 1) << 1) | ((c >> bit) & 1)
                r |= ((imm >> idx) & 1) << bit
            wr(op[1], r)
        elif o == "v_xor_b32":
            wr(op[1], v(op[2]) ^ v(op[3]))
        elif o == "v_add_u32":
            wr(op[1], (v(op[2]) + v(op[3])) & M32)
        elif o == "v_perm_b32":   # D.byte[i] = byte sel.byte[i] of {S0:S1} (0-3: S1, 4-7: S0; 12: 0x00)
            cat = ((v(op[2]) << 32) | v(op[3])).to_bytes(8, "little")
            sel = v(op[4]).to_bytes(4, "little")
            assert all(x < 8 or x == 12 for x in sel), "v_perm selector outside the emulated subset"
            wr(op[1], int.from_bytes(bytes(cat[x] if x < 8 else 0 for x in sel), "little"))
        elif o == "ds_write_b128":
            base, off = op[1], op[2]
            for j in range(4):
                lds[addr + off + 4 * j] = v(f"v{base + j}")
        elif o == "ds_read_b128":
            q, off = op[1], op[2]
            rs = [ring_reg(q, j) for j in range(4)]
            for x in rs:
                for prs, _, _ in pending:
                    assert x not in prs, f"ds_read into {x} while it is in flight"
            # (an address nothing wrote reads as garbage: a prefetch past the last block, never consumed)
            pending.append((rs, [lds.get(addr + off + 4 * j, 0xBAD0BAD0) for j in range(4)],
                            [addr + off + 4 * j for j in range(4)]))
        elif o == "s_waitcnt_lgkm":
            while len(pending) > op[1]:
                rs, vals, _ = pending.pop(0)
                for x, val in zip(rs, vals):
                    regs[x] = val
        elif o == "s_barrier":
            if on_barrier is not None:
                on_barrier({a for _, _, adrs in pending for a in adrs})
        elif o == "s_nop":
            pass
        else:
            raise ValueError(o)
    if drain:
        assert not pending, "ds_read still in flight at the end of the block"
    return regs


def emulate_twin(ins, regs2, lds, addrs, on_barrier=None, pend=None, drain: bool = True):
    """Run an instruction list on the two lanes of a TWIN pair in lockstep (regs2 / addrs per lane).
    v_add_u32_dpp reads its first source from the owning lane (op[4]); every other instruction runs per
    lane through emulate(), with each lane's in-flight reads carried across instructions."""
    pend = pend if pend is not None else ([], [])
    for op in ins:
        if op[0] == "v_add_u32_dpp":
            _, dst, src, src1, b = op
            vals = []
            for ln in range(2):
                assert all(src not in rs for rs, _, _ in pend[b]), f"DPP read of {src} in flight"
                assert all(src1 not in rs and dst not in rs for rs, _, _ in pend[ln]), "in-flight register"
                vals.append((regs2[b][src] + regs2[ln][src1]) & M32)
            for ln in range(2):
                regs2[ln][dst] = vals[ln]
        elif op[0] == "s_barrier":
            if on_barrier is not None:
                on_barrier({a for ln in range(2) for _, _, adrs in pend[ln] for a in adrs})
        else:
            for ln in range(2):
                emulate([op], regs2[ln], lds, addrs[ln], drain=False, pending=pend[ln])
    if drain:
        assert not pend[0] and not pend[1], "ds_read still in flight at the end of the block"
    return regs2


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
    # HELPER: raw little-endian words -> K+W[0..79] in LDS
    regs = {"sel": 0x00010203}
    regs.update({f"k{i}": K[i] for i in range(4)})
    regs.update({f"raw{i}": int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)})
    lds = {}
    emulate(gen_helper(), regs, lds, 0)
    for t in range(80):
        assert lds[1024 * (t // 4) + 4 * (t % 4)] == (ww[t] + (0 if K_IN_ROUNDS else K[t // 20])) & M32, \
            "SHA1_HELPER mismatch"
    # LDS rounds consume the helper's output
    regs = dict(base)
    emulate(gen_lds(), regs, lds, 0)
    got = [(h[i] + regs[f"r{i}"]) & M32 for i in range(5)]
    assert got == exp, "SHA1_LDS mismatch"
    # TWIN: the helper's twin layout for piece 33 (helper lane 33; rounds wave 1, lanes 2 and 3)
    if not K_IN_ROUNDS:
        hregs = []
        for ln in range(2):
            regs = {"sel": 0x00010203, "psel": (0x03020100, 0x07060504)[ln]}
            regs.update({f"k{i}": K[i] for i in range(4)})
            regs.update({f"raw{i}": int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)})
            hregs.append(regs)
        lds = {}
        # piece 33: lanes 2 and 3 of wave 1 (helper wave 3 writes where rounds wave 1 reads)
        emulate_twin(gen_helper2(), hregs, lds, [1024 + 2 * 16, 1024 + 3 * 16])
        for t in range(80):
            a = 1024 + (t // 8) * TWIN_READ_BYTES + (2 + t % 2) * 16 + 4 * ((t % 8) // 2)
            assert lds[a] == (ww[t] + K[t // 20]) & M32, "SHA1_HELPER2 mismatch"
        regs2 = [dict(base), dict(base)]
        emulate_twin(gen_twin(0, lead=True), regs2, lds, [1024 + 2 * 16, 1024 + 3 * 16])
        for ln in range(2):
            got = [(h[i] + regs2[ln][f"r{i}"]) & M32 for i in range(5)]
            assert got == exp, f"SHA1_TWIN mismatch (lane {ln})"
    return exp


def _kw_words(block: bytes):
    def rotl(x, n):
        return ((x << n) | (x >> (32 - n))) & M32
    ww = list(struct.unpack(">16I", block)) + [0] * 64
    for t in range(16, 80):
        ww[t] = rotl(ww[t - 3] ^ ww[t - 8] ^ ww[t - 14] ^ ww[t - 16], 1)
    return [(ww[t] + (0 if K_IN_ROUNDS else K[t // 20])) & M32 for t in range(80)]


def check_rounds_stream(blocks, h):
    """The pipelined rounds stream over consecutive blocks, run exactly as rounds_loop_text lays it out
    (prologue, blocks on buffers 0, 1, 2, 0, ...), against the helper's protocol: blocks 0 and 1 are in
    LDS at the start; at the barrier that ends block k (B_{k+1}) block k+3's buffer is poisoned (the real
    helper may be writing it from then on) and block k+2 is written (the latest moment the protocol
    allows).  A read of a block too early, or of a buffer after it was handed back, returns wrong words."""
    lds = {}

    def put(m, words, in_flight=frozenset()):
        base = (m % LDS_BUFS) * RING_BYTES
        for t in range(80):
            a = base + 1024 * (t // 4) + 4 * (t % 4)
            assert a not in in_flight, f"LDS {a} rewritten while a ds_read of it is in flight"
            lds[a] = words[t]

    kws = [_kw_words(b) for b in blocks]
    put(0, kws[0])
    if len(blocks) > 1:
        put(1, kws[1])
    state = {"k": 0}

    def on_barrier(in_flight):
        k = state["k"]               # the block that just ended
        state["k"] = k + 1
        put(k + 3, [0xDEADBEEF ^ t for t in range(80)], in_flight)   # handed back to the helper
        if k + 2 < len(blocks):
            put(k + 2, kws[k + 2], in_flight)

    regs = {f"h{i}": h[i] for i in range(5)}
    ins = list(rounds_prologue(0))
    for k in range(len(blocks)):
        ins += gen_rounds_block((k % LDS_BUFS) * RING_BYTES, ((k + 1) % LDS_BUFS) * RING_BYTES)
    ins.append(("s_waitcnt_lgkm", 0))
    emulate(ins, regs, lds, 0, on_barrier=on_barrier)
    return [regs[f"h{i}"] for i in range(5)]


def check_split_mid_stream(blocks, h, pre: bool = False):
    """The split rounds loop with SPLIT_MID (gen_split_mid_block) or SPLIT_PRE (gen_split_pre_block, pre=True),
    checked like check_rounds_stream."""
    lds = {}

    def put(m, words, in_flight=frozenset()):
        base = (m % LDS_BUFS) * RING_BYTES
        for t in range(80):
            a = base + 1024 * (t // 4) + 4 * (t % 4)
            assert a not in in_flight, f"LDS {a} rewritten while a ds_read of it is in flight"
            lds[a] = words[t]

    kws = [_kw_words(b) for b in blocks]
    put(0, kws[0])
    if len(blocks) > 1:
        put(1, kws[1])
    state = {"k": 0}

    def on_barrier(in_flight):
        k = state["k"]
        state["k"] = k + 1
        put(k + 3, [0xDEADBEEF ^ t for t in range(80)], in_flight)
        if k + 2 < len(blocks):
            put(k + 2, kws[k + 2], in_flight)

    regs = {f"h{i}": h[i] for i in range(5)}
    ins = [("ds_read_b128", q, q * 1024) for q in range(READ_AHEAD if pre else 10)]
    for k in range(len(blocks)):
        ins += (gen_split_pre_block if pre else gen_split_mid_block)((k % LDS_BUFS) * RING_BYTES,
                                                                     ((k + 1) % LDS_BUFS) * RING_BYTES)
    ins.append(("s_waitcnt_lgkm", 0))
    emulate(ins, regs, lds, 0, on_barrier=on_barrier)
    return [regs[f"h{i}"] for i in range(5)]


def check_twin_stream(blocks, h):
    """The TWIN rounds loop over consecutive blocks as twin_rounds_loop_text lays it out, for the lane pair
    of piece 0, against the helper protocol (as check_rounds_stream): at the barrier ending block k, block
    k+3's buffer is poisoned and block k+2 written; a read in flight there must not be rewritten."""
    lds = {}

    def put(m, words, in_flight=frozenset()):
        base = (m % LDS_BUFS) * RING_BYTES
        for t in range(80):
            a = base + (t // 8) * TWIN_READ_BYTES + (t % 2) * 16 + 4 * ((t % 8) // 2)
            assert a not in in_flight, f"LDS {a} rewritten while a ds_read of it is in flight"
            lds[a] = words[t]

    kws = [_kw_words(b) for b in blocks]
    put(0, kws[0])
    if len(blocks) > 1:
        put(1, kws[1])
    state = {"k": 0}

    def on_barrier(in_flight):
        k = state["k"]
        state["k"] = k + 1
        put(k + 3, [0xDEADBEEF ^ t for t in range(80)], in_flight)
        if k + 2 < len(blocks):
            put(k + 2, kws[k + 2], in_flight)

    regs2 = [{f"h{i}": h[i] for i in range(5)} for _ in range(2)]
    ins = [("ds_read_b128", k, k * TWIN_READ_BYTES) for k in range(10)] if TWIN_PRE else []
    for k in range(len(blocks)):
        if TWIN_PRE:
            ins += gen_twin((k % LDS_BUFS) * RING_BYTES, reads_next=((k + 1) % LDS_BUFS) * RING_BYTES)
        else:
            ins += gen_twin((k % LDS_BUFS) * RING_BYTES, lead=True)
        ins += [("v_add_u32", f"h{i}", f"h{i}", f"r{i}") for i in range(5)] + [("s_barrier",)]
    ins.append(("s_waitcnt_lgkm", 0))
    emulate_twin(ins, regs2, lds, [0, 16], on_barrier=on_barrier)
    assert all(regs2[0][f"h{i}"] == regs2[1][f"h{i}"] for i in range(5)), "twin lanes disagree"
    return [regs2[0][f"h{i}"] for i in range(5)]


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
    # the split kernel's pipelined rounds stream over 1 .. 7 consecutive blocks (every buffer phase)
    for n in ([0, 55, 64, 119, 200, 310, 400] if PIPELINED else []):
        msg = bytes(rng.randrange(256) for _ in range(n))
        padded = msg + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
        h0 = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        h = check_rounds_stream([padded[i:i + 64] for i in range(0, len(padded), 64)], h0)
        assert struct.pack(">5I", *h) == hashlib.sha1(msg).digest(), ("stream", n)
    # the split rounds loop with the next block's reads issued mid-block, 1 .. 7 blocks
    for n in ([0, 55, 64, 119, 200, 310, 400] if SPLIT_MID else []):
        msg = bytes(rng.randrange(256) for _ in range(n))
        padded = msg + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
        h0 = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        h = check_split_mid_stream([padded[i:i + 64] for i in range(0, len(padded), 64)], h0)
        assert struct.pack(">5I", *h) == hashlib.sha1(msg).digest(), ("split mid stream", n)
    for n in ([0, 55, 64, 119, 200, 310, 400] if SPLIT_PRE else []):
        msg = bytes(rng.randrange(256) for _ in range(n))
        padded = msg + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
        h0 = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        h = check_split_mid_stream([padded[i:i + 64] for i in range(0, len(padded), 64)], h0, pre=True)
        assert struct.pack(">5I", *h) == hashlib.sha1(msg).digest(), ("split pre stream", n)
    # the TWIN rounds loop over 1 .. 7 consecutive blocks (every buffer phase)
    for n in ([0, 55, 64, 119, 200, 310, 400] if LDS_BUFS == 3 and not K_IN_ROUNDS else []):
        msg = bytes(rng.randrange(256) for _ in range(n))
        padded = msg + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
        h0 = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        h = check_twin_stream([padded[i:i + 64] for i in range(0, len(padded), 64)], h0)
        assert struct.pack(">5I", *h) == hashlib.sha1(msg).digest(), ("twin stream", n)
    return True


# ---------------------------------------------------------------- emitter --------------

def _opnd(x, full: bool):
    if isinstance(x, int):
        return str(x)
    if x.startswith("v") and x[1:].isdigit():
        return x  # physical ring register
    return f"%[{x}]"


def _emit_lines(ins, full: bool = False):
    lines = []
    for op in ins:
        o = op[0]
        if o == "s_waitcnt_lgkm":
            lines.append(f"s_waitcnt lgkmcnt({op[1]})")
        elif o == "ds_read_b128":
            q, off = op[1], op[2]
            lo = RING_BASE + 4 * (q % RING_QUADS)
            a, off = ("%[addr2]", off - 65536) if off >= 65536 else ("%[addr]", off)   # (16-bit DS offsets)
            lines.append(f"ds_read_b128 v[{lo}:{lo + 3}], {a} offset:{off}")
        elif o == "v_bitop3_b32":
            lines.append(f"v_bitop3_b32 {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}, "
                         f"{_opnd(op[4], full)} bitop3:0x{op[5]:02x}")
        elif o == "v_alignbit_b32":
            lines.append(f"v_alignbit_b32 {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}, {op[4]}")
        elif o in ("v_xor_b32", "v_add_u32"):
            lines.append(f"{o} {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}")
        elif o == "v_perm_b32":
            lines.append(f"v_perm_b32 {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)}, {_opnd(op[4], full)}")
        elif o == "ds_write_b128":
            a, off = ("%[addr2]", op[2] - 65536) if op[2] >= 65536 else ("%[addr]", op[2])
            lines.append(f"ds_write_b128 {a}, v[{op[1]}:{op[1] + 3}] offset:{off}")
        elif o == "s_barrier":
            lines.append("s_barrier")
        elif o == "s_nop":
            lines.append("s_nop 0")
        elif o == "v_add_u32_dpp":
            b = op[4]
            lines.append(f"v_add_u32_dpp {_opnd(op[1], full)}, {_opnd(op[2], full)}, {_opnd(op[3], full)} "
                         f"quad_perm:[{b},{b},{2 + b},{2 + b}] row_mask:0xf bank_mask:0xf")
        else:
            lines.append(f"{o} " + ", ".join(_opnd(x, full) for x in op[1:]))
    return lines


def emit(ins, full: bool) -> str:
    return "\n".join(f'    "{l}\\n"' for l in _emit_lines(ins, full))


HEADER = """// GENERATED by tools/gen_sha1_asm.py -- do not edit.  Regenerate with:
//   python3 tools/gen_sha1_asm.py
// The instruction streams below are checked against hashlib by the generator's emulator
// (tests/test_abi.py::test_asm_generator_emulator) before they are written.
#pragma once
#include <stdint.h>

#define TV_SHA1_RING_BASE {ring_base}
#define TV_SHA1_RING_QUADS {ring_quads}
// K+W buffers per split-kernel pair, and how many blocks the helper wave runs ahead of the rounds wave
// (its first HELPER_AHEAD - 1 writes are not followed by a barrier; it ends with as many extra barriers)
#define TV_SHA1_LDS_BUFS {lds_bufs}
#define TV_SHA1_HELPER_AHEAD {helper_ahead}
// 1: the split helper writes W and the rounds wave adds K (v_add3 with an SGPR); 0: the helper writes K+W
#define TV_SHA1_K_IN_ROUNDS {k_in_rounds}

// One SHA-1 compression, schedule in-asm.  w[16] holds the big-endian message words and is
// clobbered.  On return r = working state after round 79; caller does h += r.
__device__ __forceinline__ void tv_sha1_full(const uint32_t h[5], uint32_t r[5], uint32_t w[16],
                                             uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t t0, t1, t2, t3;
    // volatile + "memory": the compiler may not move the caller's prefetch loads across the block
    // (otherwise it sinks them next to their use and the load latency is exposed every block).
    asm volatile(
{full}
    : [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [w0] "+v"(w[0]), [w1] "+v"(w[1]), [w2] "+v"(w[2]), [w3] "+v"(w[3]),
      [w4] "+v"(w[4]), [w5] "+v"(w[5]), [w6] "+v"(w[6]), [w7] "+v"(w[7]),
      [w8] "+v"(w[8]), [w9] "+v"(w[9]), [w10] "+v"(w[10]), [w11] "+v"(w[11]),
      [w12] "+v"(w[12]), [w13] "+v"(w[13]), [w14] "+v"(w[14]), [w15] "+v"(w[15]),
      [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
    : [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]), [h4] "v"(h[4]),
      [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : "memory");
}}

// The 80 rounds of one compression with K+W[0..79] read from LDS at byte address `addr`
// (+ g*1024 for quad g), as written by tv_sha1_schedule_lds.  Waits for all of its own LDS reads
// before returning.
__device__ __forceinline__ void tv_sha1_lds(const uint32_t h[5], uint32_t r[5], uint32_t addr,
                                            uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t t0, t1;
    asm volatile(
{lds}
    : [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [t0] "=&v"(t0), [t1] "=&v"(t1)
    : [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]), [h4] "v"(h[4]), [addr] "v"(addr){addr2},
      [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {ring_clobbers}, "memory");
}}

// The split kernel's helper wave over its nraw (>= 1) raw blocks: va = address of the first
// block of this lane's piece, addr = LDS byte address of this lane in ring buffer 0.  One
// workgroup barrier per block (matching the rounds wave).  Returns with no load in flight.
__device__ __forceinline__ void tv_sha1_helper_loop(const void* va, uint32_t nraw, uint32_t addr,
                                                    uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t cnt, adv;
    uint64_t inc;
    asm volatile(
{helper_loop}
    : [cnt] "=&s"(cnt), [adv] "=&s"(adv), [inc] "=&s"(inc)
    : [va] "v"(va), [nraw] "s"(nraw), [addr] "v"(addr){addr2}, [sel] "s"(0x00010203u),
      [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {loop_clobbers}, "scc", "memory");
}}

// The split kernel's rounds wave over nsteps (>= 1) consecutive blocks starting with ring buffer 0,
// in which every lane updates its chaining value: 80 rounds from LDS, h += r, workgroup barrier.
__device__ __forceinline__ void tv_sha1_rounds_loop(uint32_t h[5], uint32_t addr, uint32_t nsteps,
                                                    uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t r[5], t0, t1, cnt;
    asm volatile(
{rounds_loop}
    : [h0] "+v"(h[0]), [h1] "+v"(h[1]), [h2] "+v"(h[2]), [h3] "+v"(h[3]), [h4] "+v"(h[4]),
      [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [t0] "=&v"(t0), [t1] "=&v"(t1), [cnt] "=&s"(cnt)
    : [addr] "v"(addr){addr2}, [nsteps] "s"(nsteps), [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {ring_clobbers}, "scc", "memory");
}}

// Message schedule of one block for the split kernel's helper wave: raw[16] are the block's words
// as loaded (little-endian); writes K+W[0..79] to LDS at `addr` (+ q*1024 for quad q).  The LDS
// writes are left in flight (the caller's barrier waits lgkmcnt(0)).
__device__ __forceinline__ void tv_sha1_schedule_lds(const uint32_t raw[16], uint32_t addr,
                                                     uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    asm volatile(
{helper}
    :
    : [raw0] "v"(raw[0]), [raw1] "v"(raw[1]), [raw2] "v"(raw[2]), [raw3] "v"(raw[3]),
      [raw4] "v"(raw[4]), [raw5] "v"(raw[5]), [raw6] "v"(raw[6]), [raw7] "v"(raw[7]),
      [raw8] "v"(raw[8]), [raw9] "v"(raw[9]), [raw10] "v"(raw[10]), [raw11] "v"(raw[11]),
      [raw12] "v"(raw[12]), [raw13] "v"(raw[13]), [raw14] "v"(raw[14]), [raw15] "v"(raw[15]),
      [addr] "v"(addr){addr2}, [sel] "s"(0x00010203u), [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {helper_clobbers}, "memory");
}}
"""


TWIN_HEADER = """
// ---- TWIN kernel: two lanes per piece in the rounds and helper waves (tools/gen_sha1_asm.py gen_twin,
// gen_helper2).  K+W buffer layout [k][wave][lane][4 words]; a lane's `addr` is ring + (wave & 1)*1024 + lane*16,
// its `psel` 0x03020100 (even lane) / 0x07060504 (odd lane).

// One block of 80 rounds for a lane pair, with its own 10 LDS reads (waits for them before returning).
__device__ __forceinline__ void tv_sha1_twin_lds(const uint32_t h[5], uint32_t r[5], uint32_t addr) {{
    uint32_t t0, t1;
    asm volatile(
{twin_lds}
    : [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [t0] "=&v"(t0), [t1] "=&v"(t1)
    : [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]), [h4] "v"(h[4]), [addr] "v"(addr){addr2}
    : {ring_clobbers}, "memory");
}}

// The TWIN rounds wave over nsteps (>= 1) blocks from ring buffer 0 in which every lane updates.
__device__ __forceinline__ void tv_sha1_twin_rounds_loop(uint32_t h[5], uint32_t addr, uint32_t nsteps) {{
    uint32_t r[5], t0, t1, cnt;
    asm volatile(
{twin_rounds_loop}
    : [h0] "+v"(h[0]), [h1] "+v"(h[1]), [h2] "+v"(h[2]), [h3] "+v"(h[3]), [h4] "+v"(h[4]),
      [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [t0] "=&v"(t0), [t1] "=&v"(t1), [cnt] "=&s"(cnt)
    : [addr] "v"(addr){addr2}, [nsteps] "s"(nsteps)
    : {ring_clobbers}, "scc", "memory");
}}

// The TWIN helper wave (64 pieces, one lane each) over its nraw (>= 1) raw blocks: as
// tv_sha1_helper_loop, writing the twin layout.
__device__ __forceinline__ void tv_sha1_twin_helper_loop(const void* va, uint32_t nraw, uint32_t addr, uint32_t psel,
                                                         uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t cnt, adv;
    uint64_t inc;
    asm volatile(
{twin_helper_loop}
    : [cnt] "=&s"(cnt), [adv] "=&s"(adv), [inc] "=&s"(inc)
    : [va] "v"(va), [nraw] "s"(nraw), [addr] "v"(addr){addr2}, [sel] "s"(0x00010203u), [psel] "v"(psel),
      [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {twin_loop_clobbers}, "scc", "memory");
}}

// Message schedule of one block into the twin layout (the helper's padded tail blocks).
__device__ __forceinline__ void tv_sha1_twin_schedule_lds(const uint32_t raw[16], uint32_t addr, uint32_t psel,
                                                          uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    asm volatile(
{twin_helper}
    :
    : [raw0] "v"(raw[0]), [raw1] "v"(raw[1]), [raw2] "v"(raw[2]), [raw3] "v"(raw[3]),
      [raw4] "v"(raw[4]), [raw5] "v"(raw[5]), [raw6] "v"(raw[6]), [raw7] "v"(raw[7]),
      [raw8] "v"(raw[8]), [raw9] "v"(raw[9]), [raw10] "v"(raw[10]), [raw11] "v"(raw[11]),
      [raw12] "v"(raw[12]), [raw13] "v"(raw[13]), [raw14] "v"(raw[14]), [raw15] "v"(raw[15]),
      [addr] "v"(addr){addr2}, [sel] "s"(0x00010203u), [psel] "v"(psel), [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : {twin_helper_clobbers}, "memory");
}}
"""


def render() -> str:
    ring = ", ".join(f'"v{RING_BASE + i}"' for i in range(4 * RING_QUADS))
    hregs = list(range(HW_BASE, HW_BASE + 16)) + [HT, HT2] + list(range(HOUT_BASE, HOUT_BASE + 4 * HOUT_QUADS))
    helper = ", ".join(f'"v{i}"' for i in hregs)
    loop = ", ".join(f'"v{i}"' for i in hregs + list(range(P0_BASE, VL + 2)))
    h2regs = list(range(H2_F, H2_O + 12))
    h2 = ", ".join(f'"v{i}"' for i in h2regs)
    h2loop = ", ".join(f'"v{i}"' for i in h2regs + list(range(P0_BASE, VL + 2)))
    # a K+W ring past 64 KiB (LDS_BUFS >= 4) addresses its upper buffers from a second register: DS offsets are 16-bit
    addr2 = ', [addr2] "v"(addr + 65536u)' if LDS_BUFS * RING_BYTES > 65536 else ""
    return HEADER.format(addr2=addr2, k_in_rounds=int(K_IN_ROUNDS), ring_base=RING_BASE, ring_quads=RING_QUADS, lds_bufs=LDS_BUFS, helper_ahead=HELPER_AHEAD,
                         full=('    ".p2align 3\\n"\n' if ALIGN_FULL else "") + emit(gen_full(), True),
                         lds=emit(gen_lds(), False), helper=emit(gen_helper(), False),
                         helper_loop=helper_loop_text(), rounds_loop=rounds_loop_text(),
                         ring_clobbers=ring, helper_clobbers=helper,
                         loop_clobbers=loop) + ("" if K_IN_ROUNDS else TWIN_HEADER.format(
                             twin_lds='    ".p2align 3\\n"\n' + emit(gen_twin(0, lead=True), False),
                             twin_rounds_loop=twin_rounds_loop_text(),
                             twin_helper_loop=helper_loop_text(twin=True),
                             twin_helper=emit(gen_helper2(), False),
                             ring_clobbers=ring, twin_helper_clobbers=h2, twin_loop_clobbers=h2loop, addr2=addr2))


def _stamp_patch(txt: str) -> str:
    """STAMP builds: give tv_sha1_rounds_loop and tv_sha1_helper_loop an accumulator argument `sbar` (cycles at
    the in-loop barriers) and the SGPRs the stamps use as clobbers."""
    assert not (PIPELINED or SPLIT_MID or SPLIT_PRE), "stamps are for the shipped per-block split rounds loop"
    for fn, sig_old, out_old in (
            ("tv_sha1_rounds_loop", "uint32_t nsteps,\n", '[cnt] "=&s"(cnt)\n'),
            ("tv_sha1_helper_loop", "uint32_t nraw, uint32_t addr,\n", '[inc] "=&s"(inc)\n'),
            ("tv_sha1_twin_rounds_loop", "uint32_t nsteps) {\n", '[cnt] "=&s"(cnt)\n'),
            ("tv_sha1_twin_helper_loop", "uint32_t addr, uint32_t psel,\n", '[inc] "=&s"(inc)\n')):
        extra = fn in ("tv_sha1_helper_loop", "tv_sha1_twin_helper_loop") and STAMP >= 2
        i = txt.index(f"void {fn}(")
        j = txt.index("\n}\n", i)
        seg = txt[i:j]
        if sig_old.endswith(") {\n"):   # (a signature ending the parameter list: add before the parenthesis)
            sig_new = sig_old[:-4] + ", uint32_t& sbar) {\n"
        else:
            sig_new = sig_old[:-2] + (", uint32_t& sbar, uint32_t& svm, uint32_t& slg,\n" if extra else ", uint32_t& sbar,\n")
        for old, new in ((sig_old, sig_new),
                         (out_old, out_old[:-1] + ', [sbar] "+s"(sbar)' + (', [svm] "+s"(svm), [slg] "+s"(slg)' if extra
                                                                          else "") + "\n"),
                         ('"scc", "memory");', '"s88", "s89", "s90", "s91", "scc", "memory");')):
            assert seg.count(old) == 1, (fn, old)
            seg = seg.replace(old, new)
        txt = txt[:i] + seg + txt[j:]
    return txt.replace("#define TV_SHA1_K_IN_ROUNDS", f"#define TV_SHA1_STAMP {STAMP}\n#define TV_SHA1_K_IN_ROUNDS", 1)


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
    if STAMP:
        txt = _stamp_patch(txt)
    with open(a.out, "w") as f:
        f.write(txt)
    print(f"wrote {a.out}: FULL {len(gen_full())} instr, LDS {len(gen_lds())} instr, "
          f"HELPER {len(gen_helper())} instr")


if __name__ == "__main__":
    sys.exit(main())
