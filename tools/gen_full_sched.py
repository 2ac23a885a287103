#!/usr/bin/env python3
"""Schedules of the full SHA-1 compression (tv_sha1_full) with the message schedule pipelined.

tools/ubench_full_variants.hip found that a lone wave loses ~5 cycles per round when the VOP3
`v_add3` e+K+W sits between the previous round's new `a` (a VOP3 result) and its rotl5, and
~1.5 when two VOP3s do; a VOP2 in that window costs nothing.  The generated FULL block of
gen_sha1_asm.gen_full computes W[u] in round u-1 with the VOP2 xor in the middle of the round.
Here word u is completed in round r(u) = u - LAG with its VOP2 xor at the head of the round
(between the previous round's result and this round's rotl5) and its xor3 one round earlier.
Each stream is executed by gen_sha1_asm's emulator against hashlib before it is returned.
"""
from __future__ import annotations

import os
import random
import struct
import sys

sys.path.insert(0, os.path.dirname(__file__))
import gen_sha1_asm as G  # noqa: E402


def gen_full_pipelined(lag: int = 1, quiet_order: str = "f_first"):
    """lag = rounds between completing W[u] and its use (1 <= lag <= 15).  Rounds without schedule
    work use `quiet_order`: "plain" [ekw, rotl5, f, rotl30, fin] or "f_first" [f, ekw, rotl5, rotl30, fin]."""
    assert 1 <= lag <= 15
    ins = []
    R = G.Regs()
    done_round = {u: u - lag for u in range(16, 80)}          # round in which W[u] is completed
    start_round = {u: done_round[u] - 1 for u in range(16, 80)}  # round of its xor3
    by_done = {r: u for u, r in done_round.items()}
    by_start = {r: u for u, r in start_round.items()}
    temps = ["t2", "t3"]
    for t in range(80):
        A, B, C, D, E = G.roles(t)
        u_done = by_done.get(t)
        u_start = by_start.get(t)
        # xor3 of the word started here; alternate temps so it never waits for the previous xor
        s1 = s2 = s3 = None
        if u_start is not None:
            tt = temps[u_start & 1]
            s1 = ("v_bitop3_b32", tt, f"w{(u_start - 3) & 15}", f"w{(u_start - 8) & 15}", f"w{(u_start - 14) & 15}", 0x96)
        if u_done is not None:
            tt = temps[u_done & 1]
            wu = f"w{u_done & 15}"
            s2 = ("v_xor_b32", wu, tt, wu)
            s3 = ("v_alignbit_b32", wu, wu, wu, 31)
        e_src = R.rd(E)
        wt = f"w{t & 15}"
        ekw = lambda: ins.append(("v_add3_u32", R.wr(E), e_src, f"k{t // 20}", wt))
        rot5 = lambda: ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        fop = lambda: ins.append(G._fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))

        def rot30():
            b_src = R.rd(B)
            ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        fin = lambda: ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
        if s2 is not None:
            # [xor_s, ekw, rot5, xor3_s, f, rot30, rotl1_s, fin]; the xor overwrites W[u-16], whose
            # last use was round u-16 (< t since t >= u - 15)
            assert t >= u_done - 15 and t > u_done - 16
            ins.append(s2)
            ekw()
            rot5()
            if s1 is not None:
                ins.append(s1)
            fop()
            rot30()
            ins.append(s3)
            fin()
        else:
            if quiet_order == "f_first":
                if s1 is not None:
                    ins.append(s1)
                fop()
                ekw()
                rot5()
                rot30()
                fin()
            else:
                ekw()
                if s1 is not None:
                    ins.append(s1)
                rot5()
                fop()
                rot30()
                fin()
    assert R.cur == [f"r{i}" for i in range(5)]
    return ins


def gen_full_kw_vop2():
    """gen_sha1_asm.gen_full with e+K+W as two VOP2 adds: kw = K + W[t] (SGPR src0), e = e + kw.  One
    more instruction per round, but no VOP3 in the e+K+W slot (tools/ubench_full_variants.hip, h/i)."""
    ins = []
    R = G.Regs()
    for t in range(80):
        A, B, C, D, E = G.roles(t)
        u = t + 1
        sched = 16 <= u < 80
        wt = f"w{t & 15}"
        wu = f"w{u & 15}"
        if sched:
            ins.append(("v_bitop3_b32", "t2", f"w{(u - 3) & 15}", f"w{(u - 8) & 15}", f"w{(u - 14) & 15}", 0x96))
        ins.append(("v_add_u32", "t3", f"k{t // 20}", wt))
        e_src = R.rd(E)
        ins.append(("v_add_u32", R.wr(E), e_src, "t3"))
        ins.append(("v_alignbit_b32", "t0", R.rd(A), R.rd(A), 27))
        if sched:
            ins.append(("v_xor_b32", wu, "t2", wu))
        ins.append(G._fop(t, "t1", R.rd(B), R.rd(C), R.rd(D)))
        b_src = R.rd(B)
        ins.append(("v_alignbit_b32", R.wr(B), b_src, b_src, 2))
        if sched:
            ins.append(("v_alignbit_b32", wu, wu, wu, 31))
        ins.append(("v_add3_u32", R.rd(E), R.rd(E), "t0", "t1"))
    assert R.cur == [f"r{i}" for i in range(5)]
    return ins


def gen_full_bswap_next():
    """gen_sha1_asm.gen_full plus the NEXT block's 16 byte swaps (v_perm x_t -> n_t, sel = 0x00010203),
    one right after each of rounds 0-15's e+K+W: tools/ubench_full_variants.hip (t) found ~5 idle
    cycles per round there that another instruction fills for free."""
    out = []
    t = -1
    for op in G.gen_full():
        out.append(op)
        if op[0] == "v_add3_u32" and op[3].startswith("k"):   # this round's e+K+W
            t += 1
            if t < 16:
                out.append(("v_perm_b32", f"n{t}", 0, f"x{t}", "sel"))
    return out


def check_bswap_next(ins, n: int = 8) -> None:
    rng = random.Random(9)
    for _ in range(n):
        x = [rng.randrange(1 << 32) for _ in range(16)]
        regs = {f"x{i}": x[i] for i in range(16)}
        regs["sel"] = 0x00010203
        block = bytes(rng.randrange(256) for _ in range(64))
        h = [rng.randrange(1 << 32) for _ in range(5)]
        w = list(struct.unpack(">16I", block))
        regs.update({f"h{i}": h[i] for i in range(5)})
        regs.update({f"k{i}": G.K[i] for i in range(4)})
        regs.update({f"w{i}": w[i] for i in range(16)})
        ref = dict(regs)
        G.emulate(ins, regs)
        G.emulate(G.gen_full(), ref)
        assert [regs[f"r{i}"] for i in range(5)] == [ref[f"r{i}"] for i in range(5)]
        assert [regs[f"n{i}"] for i in range(16)] == [int.from_bytes(v.to_bytes(4, "little"), "big") for v in x]


def check(ins, n: int = 20) -> None:
    rng = random.Random(7)
    for _ in range(n):
        block = bytes(rng.randrange(256) for _ in range(64))
        h = [rng.randrange(1 << 32) for _ in range(5)]
        w = list(struct.unpack(">16I", block))
        regs = {f"h{i}": h[i] for i in range(5)}
        regs.update({f"k{i}": G.K[i] for i in range(4)})
        regs.update({f"w{i}": w[i] for i in range(16)})
        G.emulate(ins, regs)
        # reference
        def rotl(x, k):
            return ((x << k) | (x >> (32 - k))) & G.M32
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
            a, b, c, d, e = (rotl(a, 5) + (f & G.M32) + e + G.K[t // 20] + ww[t]) & G.M32, a, rotl(b, 30), c, d
        got = [regs[f"r{i}"] for i in range(5)]
        assert got == [a, b, c, d, e], "schedule variant computes a wrong state"


if __name__ == "__main__":
    check(gen_full_kw_vop2())
    check_bswap_next(gen_full_bswap_next())
    print("bswap_next:", len(gen_full_bswap_next()), "instr ok")
    print("kw_vop2:", len(gen_full_kw_vop2()), "instr ok")
    for lag in (1, 2, 3):
        for q in ("plain", "f_first"):
            ins = gen_full_pipelined(lag, q)
            check(ins)
            print(f"lag {lag} quiet {q}: {len(ins)} instr ok")
