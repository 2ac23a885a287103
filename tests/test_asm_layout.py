"""Instruction layout of the SHA-1 hot loops (CPU only).

A lone wave issues long runs of 8-byte instructions placed at 4 mod 8 at ~5.07 instead of 4.07 cycles each
(tools/gen_ubench_align.py), which cost the lane kernel 4.7 % at cfg4 before the
generator paired the schedule's 4-byte xors and aligned the block.  These tests keep that layout:
  * the generated lane compression (tv_sha1_full) starts with .p2align 3 and keeps every 8-byte VOP3 at an
    8-byte offset from its start;
  * in the built library, the lane kernel's main loop has almost no misaligned 8-byte instructions, the
    split kernel's rounds loop no misaligned run longer than five (runs up to five are free), and the twin
    kernel's rounds loop (five 8-byte instructions per round) none at all and no padding s_nop, its head at
    4 mod 64 and its helper loop's at 60 mod 64 (the 64-byte placement is worth ~1 % at cfg2).
"""
import os
import re
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HEADER = os.path.join(ROOT, "torrent_amd", "csrc", "sha1_asm.h")
LIB = os.path.join(ROOT, "torrent_amd", "libtorrent_verify.so")

SIZE = {"v_add3_u32": 8, "v_alignbit_b32": 8, "v_bitop3_b32": 8, "v_perm_b32": 8,
        "v_xor_b32": 4, "v_add_u32": 4}


def _full_block():
    txt = open(HEADER).read()
    body = txt[txt.index("void tv_sha1_full("):]
    body = body[body.index("asm volatile("):body.index("    : [r0]")]
    return re.findall(r'"([^"\\]+)\\n"', body)


def test_lane_compression_block_is_8_byte_aligned():
    lines = _full_block()
    assert lines[0] == ".p2align 3"
    off = 0
    for l in lines[1:]:
        op = l.split()[0]
        size = SIZE[op]
        if size == 8:
            assert off % 8 == 0, f"{l!r} at block offset {off}"
        off += size
    assert off % 8 == 0
    # the 64 schedule xors come in adjacent pairs
    ops = [l.split()[0] for l in lines[1:]]
    xs = [i for i, o in enumerate(ops) if o == "v_xor_b32"]
    assert len(xs) == 64 and all(xs[k + 1] == xs[k] + 1 for k in range(0, 64, 2))


@pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and llvm-objdump")
def test_built_hot_loops_alignment():
    from tools.asm_alignment import analyze
    rep = analyze(LIB)
    main = [r for r in rep["lane"] if r["instrs"] >= 1500]     # the 3-block unrolled raw-block loop
    assert main, rep["lane"]
    for r in main:
        assert r["misaligned"] <= 0.03 * r["eight_byte"], r
    rounds = [r for r in rep["split"] if r["instrs"] >= 1200 and r["eight_byte"] > 0.7 * r["instrs"]]
    assert rounds, rep["split"]
    for r in rounds:
        assert max(int(k) for k in r["runs"]) <= 5, r
    # the twin rounds loop (3 blocks of 80 five-instruction rounds, all 8-byte): fully aligned, and no s_nop
    twin = [r for r in rep["twin"] if r["instrs"] >= 1000 and r["eight_byte"] > 0.9 * r["instrs"]]
    assert twin, rep["twin"]
    for r in twin:
        assert r["misaligned"] == 0 and r["s_nop"] == 0, r
        # pinned at 4 mod 64 (1 % faster at cfg2 than where the code before it happened to put it in round 3:
        # profiles/r03/twin_ralign.jsonl)
        assert int(r["first"], 16) % 64 == 4, r
    # the twin helper loop (3 blocks, ~350 instructions) pinned at 60 mod 64
    helper = [r for r in rep["twin"] if 300 <= r["instrs"] <= 400]
    assert helper and all(int(r["first"], 16) % 64 == 60 for r in helper), rep["twin"]
