#!/usr/bin/env python3
"""Write tools/ubench_rounds.hip (generated on demand, not committed): the split kernel's rounds block (gen_sha1_asm.gen_lds) in a loop
on one wave per CU, with variants of how K+W arrives from LDS.

Question: the rounds wave runs 1,952 cyc per block, but 80 rounds of the same VALU mix in a loop
with no LDS run at ~1,635 (tools/ubench_fetch.hip).  Where do the other ~300 cycles go, and which
LDS read shape costs least?  Variants (same 400-VALU round stream each):
  real     the generated block: 20 ds_read_b128, 7 quads ahead, one lgkmcnt wait per 4 quads
  nolds    no LDS reads and no waits (K+W from stale registers): the VALU floor
  nowait   the reads, but no waits inside the block (one wait at the end)
  b64      40 ds_read_b64 instead of 20 ds_read_b128 (waits scaled)
  late     each ds_read_b128 issued after the round's add3 instead of after its first add
  hadd     real + the 5 `h += r` adds and s_barrier of the kernel's loop
Build: python3 tools/gen_ubench_rounds.py && hipcc --offload-arch=gfx950 -O3 tools/ubench_rounds.hip -o tools/ubench_rounds
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


def variant(name: str) -> list[str]:
    rq, ra, we = SWEEP.get(name, (8, 7, 4))
    g.RING_QUADS, g.READ_AHEAD, g.WAIT_EVERY = rq, ra, we
    ins = g.gen_lds(0, lead_wait=False)
    out = []
    if name == "late":
        pending = None
        for op in ins:
            if op[0] == "ds_read_b128" and any(x[0].startswith("v_") for x in out):
                pending = op
                continue
            out.append(op)
            if op[0] == "v_add3_u32" and pending is not None:
                out.append(pending)
                pending = None
        ins = out
        out = []
    for line in g._emit_lines(ins):
        line = phys(line)
        if name == "nolds" and (line.startswith("ds_read") or line.startswith("s_waitcnt")):
            continue
        if name == "nowait" and line.startswith("s_waitcnt"):
            continue
        if name in ("kadd3", "kadd3v") and line.startswith("v_add_u32"):
            # e + K + W as one v_add3 with K in an SGPR (kadd3) or a VGPR (kadd3v), W from the ring
            m = re.match(r"v_add_u32 (v\d+), (v\d+), (v\d+)", line)
            k = "s44" if name == "kadd3" else "v47"
            out.append(f"v_add3_u32 {m.group(1)}, {m.group(3)}, {k}, {m.group(2)}")
            continue
        if name == "b64" and line.startswith("ds_read_b128"):
            m = re.match(r"ds_read_b128 v\[(\d+):(\d+)\], (v\d+) offset:(\d+)", line)
            lo, addr, off = int(m.group(1)), m.group(3), int(m.group(4))
            out.append(f"ds_read_b64 v[{lo}:{lo + 1}], {addr} offset:{off}")
            out.append(f"ds_read_b64 v[{lo + 2}:{lo + 3}], {addr} offset:{off + 8}")
            continue
        if name == "b64" and line.startswith("s_waitcnt"):
            n = int(re.search(r"\((\d+)\)", line).group(1))
            out.append(f"s_waitcnt lgkmcnt({min(15, 2 * n)})")
            continue
        out.append(line)
    if name in ("hadd", "pair_rounds"):
        out += [f"v_add_u32 v{50 + i}, v{50 + i}, v{40 + i}" for i in range(5)] + ["s_barrier"]
    out.append("s_waitcnt lgkmcnt(0)")
    return out


# ring quads, quads read ahead, quads per lgkmcnt wait (the generator's RING_QUADS / READ_AHEAD / WAIT_EVERY)
SWEEP = {"q8a7w2": (8, 7, 2), "q8a7w1": (8, 7, 1), "q8a4w4": (8, 4, 4), "q8a6w2": (8, 6, 2),
         "q16a15w8": (16, 15, 8), "q16a12w4": (16, 12, 4), "q16a15w4": (16, 15, 4), "q16a8w8": (16, 8, 8)}
VARIANTS = ["real", "nolds", "nowait", "b64", "late", "hadd"] + list(SWEEP)
SWEEP["pair_rounds"] = (16, 15, 4)
SWEEP["kadd3"] = SWEEP["kadd3v"] = (16, 15, 4)
VARIANTS += ["kadd3", "kadd3v"]
PAIR_HELPERS = {"pair_bar": (0, 0), "pair_valu": (0, 300), "pair_wr": (20, 0), "pair_full": (20, 300),
                "pair_vop2": (20, 300), "pair_prio": (20, 300), "pair_half": (20, 140)}


def render() -> str:
    clob = ", ".join(f'"v{r}"' for r in list(range(40, 56)) + list(range(60, 128)))
    kern = []
    for vi, name in enumerate(VARIANTS):
        body = "\n".join(f'        "{l}\\n"' for l in variant(name))
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
        "s_branch L_top_%=\\n"
        ".p2align 6\\n"
        "L_top_%=:\\n"
{body}
        "s_sub_u32 s40, s40, 1\\n"
        "s_cmp_lg_u32 s40, 0\\n"
        "s_cbranch_scc1 L_top_%=\\n"
        "v_mov_b32 %0, v40\\n"
        : "=v"(o) : "v"(addr), "v"(a) : "s40", "scc", "memory", {clob});
    asm volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = o + lds[threadIdx.x];
}}""")
    # two-wave workgroups: wave 0 = the rounds block (16-quad ring) + 5 adds + s_barrier per block;
    # wave 1 = a helper stand-in per block: PAIR_HELPERS[name] = (ds_write_b128 count, VALU count)
    rounds = variant("pair_rounds")
    for name, (nw, nv) in PAIR_HELPERS.items():
        hb = []
        for q in range(20):
            op = "v_xor_b32 v60, v61, v62" if name == "pair_vop2" else "v_bitop3_b32 v60, v61, v62, v63 bitop3:0x96"
            hb += [op] * (nv // 20)
            if q < nw:
                hb.append(f"ds_write_b128 v49, v[64:67] offset:{20480 + q * 1024}")
        hb += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
        rl = (["s_setprio 3"] if name == "pair_prio" else []) + rounds
        rbody = "\n".join(f'            "{l}\\n"' for l in rl)
        hbody = "\n".join(f'            "{l}\\n"' for l in hb)
        kern.append(f"""
__global__ __launch_bounds__(128) void k_{name}(uint64_t* cyc, uint32_t* sink, uint32_t seed) {{
    __shared__ uint32_t lds[40 * 256 + 64];
    for (int i = threadIdx.x; i < 40 * 256 + 64; i += 128) lds[i] = i * seed;
    __syncthreads();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t addr = (threadIdx.x & 63) * 16, a = threadIdx.x ^ seed, o = 0;
    uint64_t t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    if (wave == 0) {{
        asm volatile(
            "v_mov_b32 v49, %1\\n v_mov_b32 v40, %2\\n v_mov_b32 v41, %2\\n v_mov_b32 v42, %2\\n"
            "v_mov_b32 v43, %2\\n v_mov_b32 v44, %2\\n s_mov_b32 s40, {NBLK}\\n s_branch L_top_%=\\n"
            ".p2align 6\\n L_top_%=:\\n"
{rbody}
            "s_sub_u32 s40, s40, 1\\n s_cmp_lg_u32 s40, 0\\n s_cbranch_scc1 L_top_%=\\n"
            "v_mov_b32 %0, v40\\n"
            : "=v"(o) : "v"(addr), "v"(a) : "s40", "scc", "memory", {clob});
    }} else {{
        asm volatile(
            "v_mov_b32 v49, %1\\n v_mov_b32 v61, %2\\n v_mov_b32 v62, %2\\n v_mov_b32 v63, %2\\n"
            "s_mov_b32 s40, {NBLK}\\n s_branch L_top_%=\\n .p2align 6\\n L_top_%=:\\n"
{hbody}
            "s_sub_u32 s40, s40, 1\\n s_cmp_lg_u32 s40, 0\\n s_cbranch_scc1 L_top_%=\\n"
            "v_mov_b32 %0, v60\\n"
            : "=v"(o) : "v"(addr), "v"(a) : "s40", "scc", "memory", {clob});
    }}
    asm volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if ((threadIdx.x & 63) == 0 && wave == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 128 + threadIdx.x] = o + lds[threadIdx.x];
}}""")
    runs = "\n".join(f'    run(k_{n}, "{n}", {128 if n in PAIR_HELPERS else 64});' for n in VARIANTS + list(PAIR_HELPERS))
    return f"""// GENERATED by tools/gen_ubench_rounds.py -- see its docstring.
#include <hip/hip_runtime.h>

#include <cstdio>
{''.join(kern)}

template <typename K>
void run(K kern, const char* name, int threads) {{
    const int blocks = 256;
    uint64_t* cyc;
    uint32_t* sink;
    (void)hipMalloc(&cyc, sizeof(uint64_t) * blocks);
    (void)hipMalloc(&sink, 4 * blocks * 128);
    double best = 1e30;
    for (int rep = 0; rep < 4; rep++) {{
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, cyc, sink, 1u);
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
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "ubench_rounds.hip"), "w") as f:
        f.write(render())
