#!/usr/bin/env python3
"""Write tools/ubench_dpp.hip (generated on demand, not committed): does sharing the K+W reads between two
lanes of a piece pay?

Idea (round 2 re-entry): the split kernel's rounds wave spends ~160 of its ~1,890 cycles per block on 20
ds_read_b128 (an issue slot each plus the 1 KiB VGPR write-back).  With TWO lanes per piece, both lanes run
the same rounds on the same data, lane 2p+0 reads the even K+W quads and lane 2p+1 the odd ones, and the
round's `e + KW` add reads the owning lane's register through DPP (quad_perm [b,b,2+b,2+b]): 10 reads per
block instead of 20, at the price of half the pieces per wave (the cfg2 grid has SIMDs to spare).  The DPP
add is an 8-byte instruction where the plain add was 4 bytes, so the round becomes five 8-byte
instructions and every 4-byte s_waitcnt flips the stream's alignment.

Variants (one lone wave per CU, NBLK blocks per loop, s_memtime cycles per block):
  base      the shipped rounds block (20 reads, 15 ahead, a wait per 4 quads) + h += r + s_barrier
  dpp20     base with every `e + KW` add as an identity-DPP add (what DPP itself costs)
  nolds     base without reads and waits (VALU floor); nolds_dpp: the same with DPP adds
  d10_*     10 reads at the block start, DPP adds; waits: w10 = one per read, w5 = one per 2 reads,
            w5n = w5 + s_nop 0 after each wait (realign), w5d = each wait doubled, w2 = waits at reads 0 and 5
Build: python3 tools/gen_ubench_dpp.py && hipcc --offload-arch=gfx950 -O3 tools/ubench_dpp.hip -o tools/ubench_dpp
"""
from __future__ import annotations

import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_sha1_asm as g  # noqa: E402

NBLK = 64
REG = {**{f"r{i}": f"v{40 + i}" for i in range(5)}, **{f"h{i}": f"v{40 + i}" for i in range(5)},
       "t0": "v45", "t1": "v46", "addr": "v49", **{f"k{i}": f"s{44 + i}" for i in range(4)}}


def phys(line: str) -> str:
    return re.sub(r"%\[(\w+)\]", lambda m: REG[m.group(1)], line)


def tail() -> list[str]:
    return [f"v_add_u32 v{50 + i}, v{50 + i}, v{40 + i}" for i in range(5)] + ["s_barrier"]


def base(dpp: bool, lds: bool = True) -> list[str]:
    g.RING_QUADS, g.READ_AHEAD, g.WAIT_EVERY = 16, 15, 4
    out = [".p2align 3"]
    for line in g._emit_lines(g.gen_lds(0, lead_wait=False)):
        line = phys(line)
        if not lds and (line.startswith("ds_read") or line.startswith("s_waitcnt")):
            continue
        if dpp and line.startswith("v_add_u32"):
            m = re.match(r"v_add_u32 (v\d+), (v\d+), (v\d+)", line)
            line = f"v_add_u32_dpp {m.group(1)}, {m.group(2)}, {m.group(3)} quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xf"
        out.append(line)
    return out + tail() + ["s_waitcnt lgkmcnt(0)"]


def d10(waits: str, pre: bool = False) -> list[str]:
    """10 ds_read_b128 at the block start (quad k of this lane = K+W quad 2k+b of its piece); round t reads
    word t%4 of read t//8 from lane b = (t//4)%2 of its pair.  pre: the reads of the NEXT block are issued
    after round 79, before h += r and the barrier (the loop prologue issues the first block's)."""
    reads = [f"ds_read_b128 v[{64 + 4 * k}:{67 + 4 * k}], v49 offset:{k * 1024}" for k in range(10)]
    out = [".p2align 3"] + ([] if pre else reads)
    nop = waits.endswith("n")
    waits = waits.rstrip("n") if waits not in ("w5n",) else "w5"
    wait_at = {"w10": range(10), "w5": range(0, 10, 2), "w5d": range(0, 10, 2),
               "w2": (0, 5), "w3": (0, 3, 6), "w1": (0,)}[waits]
    R = g.Regs()
    for t in range(80):
        k, b = t // 8, (t // 4) % 2
        if t % 8 == 0 and k in wait_at:
            nxt = [x for x in wait_at if x > k]
            need = (nxt[0] - 1) if nxt else 9            # reads consumed before the next wait
            out.append(f"s_waitcnt lgkmcnt({9 - need})")
            if waits == "w5d":
                out.append(f"s_waitcnt lgkmcnt({9 - need})")
            if nop:
                out.append("s_nop 0")
        A, B, C, D, E = g.roles(t)
        e_src = R.rd(E)
        dst = R.wr(E)
        out.append(phys(f"v_add_u32_dpp %[{dst}], v{64 + 4 * k + t % 4}, %[{e_src}] "
                        f"quad_perm:[{b},{b},{2 + b},{2 + b}] row_mask:0xf bank_mask:0xf"))
        out.append(phys(f"v_alignbit_b32 %[t0], %[{R.rd(A)}], %[{R.rd(A)}], 27"))
        op = g._fop(t, "t1", R.rd(B), R.rd(C), R.rd(D))
        out.append(phys(f"v_bitop3_b32 %[t1], %[{op[2]}], %[{op[3]}], %[{op[4]}] bitop3:0x{op[5]:02x}"))
        b_src = R.rd(B)
        out.append(phys(f"v_alignbit_b32 %[{R.wr(B)}], %[{b_src}], %[{b_src}], 2"))
        out.append(phys(f"v_add3_u32 %[{R.rd(E)}], %[{R.rd(E)}], %[t0], %[t1]"))
    if pre:
        out += reads
    return out + tail() + ([] if pre else ["s_waitcnt lgkmcnt(0)"])


VARIANTS = {
    "base": lambda: base(False), "dpp20": lambda: base(True),
    "nolds": lambda: base(False, lds=False), "nolds_dpp": lambda: base(True, lds=False),
    "d10_w10": lambda: d10("w10"), "d10_w5": lambda: d10("w5"), "d10_w5n": lambda: d10("w5n"),
    "d10_w5d": lambda: d10("w5d"), "d10_w2": lambda: d10("w2"),
    "d10_w2n": lambda: d10("w2n"), "d10_w3n": lambda: d10("w3n"), "d10_w1n": lambda: d10("w1n"),
    "pre_w5n": lambda: d10("w5n", True), "pre_w2n": lambda: d10("w2n", True), "pre_w1n": lambda: d10("w1n", True),
    "pre_w1": lambda: d10("w1", True),
}
PRE = {n for n in VARIANTS if n.startswith("pre_")}


def render() -> str:
    clob = ", ".join(f'"v{r}"' for r in list(range(40, 56)) + list(range(60, 128)))
    kern = []
    for name, fn in VARIANTS.items():
        body = "\n".join(f'        "{l}\\n"' for l in fn())
        prologue = "\n".join(f'        "ds_read_b128 v[{64 + 4 * k}:{67 + 4 * k}], v49 offset:{k * 1024}\\n"'
                             for k in range(10)) if name in PRE else ""
        kern.append(f"""
__global__ __launch_bounds__(64) void k_{name}(uint64_t* cyc, uint32_t* sink, uint32_t seed) {{
    __shared__ uint32_t lds[20 * 256 + 64];
    for (int i = threadIdx.x; i < 20 * 256 + 64; i += 64) lds[i] = i * seed;
    __syncthreads();
    uint32_t addr = threadIdx.x * 16, a = threadIdx.x ^ seed, o;
    uint64_t t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile(
        "v_mov_b32 v49, %1\\n v_mov_b32 v40, %2\\n v_mov_b32 v41, %2\\n v_mov_b32 v42, %2\\n"
        "v_mov_b32 v43, %2\\n v_mov_b32 v44, %2\\n"
        "s_mov_b32 s40, {NBLK}\\n"
{prologue}
        "s_branch L_top_%=\\n"
        ".p2align 6\\n"
        "L_top_%=:\\n"
{body}
        "s_sub_u32 s40, s40, 1\\n"
        "s_cmp_lg_u32 s40, 0\\n"
        "s_cbranch_scc1 L_top_%=\\n"
        "s_waitcnt lgkmcnt(0)\\n v_mov_b32 %0, v40\\n"
        : "=v"(o) : "v"(addr), "v"(a) : "s40", "scc", "memory", {clob});
    asm volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = o + lds[threadIdx.x];
}}""")
    runs = "\n".join(f'    run(k_{n}, "{n}");' for n in VARIANTS)
    return f"""// GENERATED by tools/gen_ubench_dpp.py -- see its docstring.
#include <hip/hip_runtime.h>

#include <cstdio>
{''.join(kern)}

template <typename K>
void run(K kern, const char* name) {{
    const int blocks = 256;
    uint64_t* cyc;
    uint32_t* sink;
    (void)hipMalloc(&cyc, sizeof(uint64_t) * blocks);
    (void)hipMalloc(&sink, 4 * blocks * 64);
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {{
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, cyc, sink, 1u);
        (void)hipDeviceSynchronize();
        uint64_t h[256];
        (void)hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; i++) s += (double)h[i];
        s /= blocks;
        if (rep && s < best) best = s;
    }}
    printf("%-10s : %7.1f cyc per block (%d blocks, one wave per CU)\\n", name, best / {NBLK}, {NBLK});
    (void)hipFree(cyc);
    (void)hipFree(sink);
}}

int main() {{
{runs}
    return 0;
}}
"""


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ubench_dpp.hip")
    with open(out, "w") as f:
        f.write(render())
    print("wrote", out)
