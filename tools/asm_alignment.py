"""Instruction-alignment report for the hot loops of the built library (a lone wave issues a long run of
8-byte instructions sitting at 4 mod 8 at ~5.07 instead of 4.07 cycles each: tools/gen_ubench_align.py,
DESIGN.md section 4).

    python tools/asm_alignment.py [path/to/libtorrent_verify.so]

Extracts the gfx950 code object with llvm-objdump --offloading (into a temporary directory), disassembles it,
and for every backward branch of the verify kernels (tv_lane_kernel<false>, tv_split_kernel<false, 1, false>,
tv_twin_kernel<false, 1>)
reports the loop's instruction count, its 8-byte instructions, how many of them sit at 4 mod 8, and the
histogram of runs of consecutive misaligned 8-byte instructions.  Prints JSON; used by tests/test_asm_layout.py.
"""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
KERNELS = {"lane": "_Z14tv_lane_kernelILb0ELb0EEv8TvPieces", "lane_pairs": "_Z14tv_lane_kernelILb0ELb1EEv8TvPieces", "split": "_Z15tv_split_kernelILb0ELi1ELb0EEv8TvPieces",
           "twin": "_Z14tv_twin_kernelILb0ELi1ELb0EEv8TvPieces"}
_INS = re.compile(r"\s+(\S.*?)\s+//\s*([0-9A-Fa-f]+):\s*((?:[0-9A-Fa-f]{8}\s*)+)")


def disassemble(so: str) -> list:
    tmp = tempfile.mkdtemp(prefix="tv_asm_")
    try:
        local = os.path.join(tmp, "lib.so")
        shutil.copy(so, local)
        subprocess.run([OBJDUMP, "--offloading", local], check=True, capture_output=True)
        objs = [f for f in os.listdir(tmp) if "gfx950" in f]
        if not objs:
            raise RuntimeError("no gfx950 code object in " + so)
        out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(tmp, objs[0])], check=True,
                             capture_output=True, text=True).stdout
        return out.splitlines()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def kernel_lines(lines: list, sym: str) -> list:
    start = next(i for i, l in enumerate(lines) if l.endswith(f"<{sym}>:"))
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <_Z", lines[i])), len(lines))
    return lines[start + 1:end]


def instrs(lines: list) -> list:
    out = []
    for l in lines:
        m = _INS.match(l)
        if m:
            out.append((int(m.group(2), 16), 4 * len(m.group(3).split()), m.group(1).split()[0]))
    return out


def loops(lines: list) -> list:
    """[(first address, backward-branch address)] of the kernel's loops, from the SOPP branch encodings
    (0xBF82 s_branch, 0xBF84..0xBF89 s_cbranch_*; simm16 = signed dword offset from the next instruction)."""
    res = []
    for l in lines:
        m = _INS.match(l)
        if not m:
            continue
        words = m.group(3).split()
        w = int(words[0], 16)
        if len(words) == 1 and (w >> 16) in (0xBF82, 0xBF84, 0xBF85, 0xBF86, 0xBF87, 0xBF88, 0xBF89):
            off = w & 0xFFFF
            if off >= 0x8000:
                addr = int(m.group(2), 16)
                res.append((addr + 4 - (0x10000 - off) * 4, addr))
    return sorted(set(res))


def report(seq: list) -> dict:
    n8 = [x for x in seq if x[1] == 8]
    mis = [x for x in n8 if x[0] % 8]
    hist, k = {}, 0
    for addr, size, _ in seq:
        if size == 8 and addr % 8:
            k += 1
        else:
            if k:
                hist[k] = hist.get(k, 0) + 1
            k = 0
    if k:
        hist[k] = hist.get(k, 0) + 1
    return {"instrs": len(seq), "eight_byte": len(n8), "misaligned": len(mis),
            "runs": {str(a): b for a, b in sorted(hist.items())}, "s_nop": sum(1 for x in seq if x[2] == "s_nop")}


def analyze(so: str) -> dict:
    lines = disassemble(so)
    out = {}
    for name, sym in KERNELS.items():
        kl = kernel_lines(lines, sym)
        all_ins = instrs(kl)
        recs = []
        for lo, hi in loops(kl):
            seq = [x for x in all_ins if lo <= x[0] <= hi]
            if len(seq) >= 200:      # the hot loops (a block or more of SHA-1), not the short control loops
                recs.append(dict(report(seq), first=hex(lo), branch=hex(hi)))
        out[name] = recs
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "torrent_amd", "libtorrent_verify.so")
    print(json.dumps(analyze(so), indent=1))


if __name__ == "__main__":
    main()
