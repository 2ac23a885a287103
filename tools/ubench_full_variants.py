#!/usr/bin/env python3
"""Writes the variants header for tools/ubench_full_variants.hip (timing-only variants a-i of the
generated tv_sha1_full, plus the pipelined schedules j-m of tools/gen_full_sched.py, which are
emulator-checked SHA-1).  usage: python3 tools/ubench_full_variants.py <out_dir>"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(__file__))
import gen_sha1_asm as G  # noqa: E402
import gen_full_sched as S  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def fn_text(name, ins):
    body = G.emit(ins, True)
    return f"""__device__ __forceinline__ void tv_sha1_full_{name}(const uint32_t h[5], uint32_t r[5], uint32_t w[16],
        uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t t0, t1, t2, t3;
    asm volatile(
{body}
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
"""


def fn_text_bswap_next(name, ins):
    body = G.emit(ins, True)
    n_out = ", ".join(f'[n{i}] "=&v"(n[{i}])' for i in range(16))
    x_in = ", ".join(f'[x{i}] "v"(x[{i}])' for i in range(16))
    return f"""__device__ __forceinline__ void tv_sha1_full_{name}(const uint32_t h[5], uint32_t r[5], uint32_t w[16],
        const uint32_t x[16], uint32_t n[16], uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {{
    uint32_t t0, t1, t2;
    asm volatile(
{body}
    : [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]), [r4] "=&v"(r[4]),
      [w0] "+v"(w[0]), [w1] "+v"(w[1]), [w2] "+v"(w[2]), [w3] "+v"(w[3]),
      [w4] "+v"(w[4]), [w5] "+v"(w[5]), [w6] "+v"(w[6]), [w7] "+v"(w[7]),
      [w8] "+v"(w[8]), [w9] "+v"(w[9]), [w10] "+v"(w[10]), [w11] "+v"(w[11]),
      [w12] "+v"(w[12]), [w13] "+v"(w[13]), [w14] "+v"(w[14]), [w15] "+v"(w[15]),
      [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), {n_out}
    : [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]), [h4] "v"(h[4]), {x_in},
      [sel] "s"(0x00010203u), [k0] "s"(k0), [k1] "s"(k1), [k2] "s"(k2), [k3] "s"(k3)
    : "memory");
}}
"""


def main(out_dir):
    src = open(os.path.join(HERE, "..", "torrent_amd", "csrc", "sha1_asm.h")).read()
    start = src.index("__device__ __forceinline__ void tv_sha1_full(")
    fn = src[start:src.index("\n}\n", start) + 3]
    var = lambda n, t: t.replace("void tv_sha1_full(", f"void tv_sha1_full_{n}(")
    vb = re.sub(r"v_bitop3_b32 (%\[t2\]), (%\[w\d+\]), (%\[w\d+\]), (%\[w\d+\]) bitop3:0x96", r"v_xor_b32 \1, \2, \3", fn)
    vc = re.sub(r"v_alignbit_b32 (%\[w\d+\]), \1, \1, 31", r"v_lshlrev_b32 \1, 1, \1", fn)
    vd = re.sub(r"v_alignbit_b32 (%\[w\d+\]), \1, \1, 31", r"v_lshlrev_b32 \1, 1, \1", vb)

    def rounds_only(t):
        t = re.sub(r'\s*"v_bitop3_b32 %\[t2\][^\n]*\n', "\n", t)
        t = re.sub(r'\s*"v_xor_b32 %\[w\d+\][^\n]*\n', "\n", t)
        return re.sub(r'\s*"v_alignbit_b32 (%\[w\d+\]), \1, \1, 31[^\n]*\n', "\n", t)
    ve = rounds_only(fn)
    kv = lambda t: re.sub(r'\[k(\d)\] "s"', r'[k\1] "v"', t)
    ekw2 = lambda t: re.sub(r"v_add3_u32 (%\[r\d\]), (%\[[rh]\d\]), %\[k\d\], (%\[w\d+\])", r"v_add_u32 \1, \2, \3", t)
    parts = [var("a", fn), var("b", vb), var("c", vc), var("d", vd), var("e", ve), var("f", kv(fn)),
             var("g", kv(ve)), var("h", ekw2(ve)), var("i", ekw2(fn))]
    # n: rounds only with e+K+W as a 2-source VOP3 (v_add_u32_e64 e, W); o: as v_add3 e, W, 0 (no SGPR);
    # p: the full block with e+K+W as v_add_u32_e64 (timing only, K dropped)
    e64 = lambda t: re.sub(r"v_add3_u32 (%\[r\d\]), (%\[[rh]\d\]), %\[k\d\], (%\[w\d+\])", r"v_add_u32_e64 \1, \2, \3", t)
    z3 = lambda t: re.sub(r"v_add3_u32 (%\[r\d\]), (%\[[rh]\d\]), %\[k\d\], (%\[w\d+\])", r"v_add3_u32 \1, \2, \3, 0", t)
    parts += [var("n", e64(ve)), var("o", z3(ve)), var("p", e64(fn))]
    # r: rounds only (e) with each e+K+W moved after the round's rotl5; s: e with s_nop 0 after each e+K+W;
    # t: e with a VOP2 v_mov (t3) after each e+K+W (timing only)
    ekw_re = r'(\s*"v_add3_u32 %\[r\d\], %\[[rh]\d\], %\[k\d\], %\[w\d+\]\\n"\n)(\s*"v_alignbit_b32 %\[t0\][^\n]*\n)'
    vr = re.sub(ekw_re, r"\2\1", ve)
    vs = re.sub(r'(\s*"v_add3_u32 %\[r\d\], %\[[rh]\d\], %\[k\d\], %\[w\d+\]\\n"\n)', r'\1    "s_nop 0\\n"\n', ve)
    vt = re.sub(r'(\s*"v_add3_u32 %\[r\d\], %\[[rh]\d\], %\[k\d\], %\[w\d+\]\\n"\n)', r'\1    "v_mov_b32 %[t2], %[t1]\\n"\n', ve)
    print("variants r/s/t:", vr.count("v_add3"), vs.count("s_nop 0"), vt.count("v_mov_b32"))
    parts += [var("r", vr), var("s", vs), var("t", vt)]
    ins_u = S.gen_full_bswap_next()
    S.check_bswap_next(ins_u)
    parts.append(fn_text_bswap_next("u", ins_u))
    ins = S.gen_full_kw_vop2()
    S.check(ins)
    parts.append(fn_text("q", ins))
    for name, (lag, q) in zip("jklm", [(1, "plain"), (1, "f_first"), (2, "f_first"), (3, "f_first")]):
        ins = S.gen_full_pipelined(lag, q)
        S.check(ins)
        parts.append(fn_text(name, ins))
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "variants.h"), "w") as f:
        f.write("#pragma once\n#include <stdint.h>\n" + "\n".join(parts))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/ubv")
