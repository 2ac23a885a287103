"""Build libtorrent_verify.so in-tree (hipcc, gfx950) -- the only native product artifact.

    python -m torrent_amd._build            # regenerate the asm header, compile the .so

The generated header torrent_amd/csrc/sha1_asm.h is produced by tools/gen_sha1_asm.py, which
first checks its instruction streams against hashlib in an emulator.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libtorrent_verify.so")
SOURCES = ["tv_kernels.hip", "tv_core.hip", "tv_context.hip", "tv_stage.hip", "tv_files.hip",
           "tv_stream.hip", "tv_verify.hip"]
HOST_SOURCES = ["tv_host.cpp"]          # host-only C++ (no device code): the host compiler
EXPORTS = os.path.join(CSRC, "exports.map")   # the link exports tv_* only
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = os.environ.get("TV_OFFLOAD_ARCH", "gfx950")


def _code_only(text: str) -> str:
    """C / C++ source without its comments and blank-line / trailing-space differences (string and character
    literals kept as they are), so that a comment or documentation edit does not change the source id."""
    out, i, n = [], 0, len(text)
    while i < n:
        c = text[i]
        if c in "\"'":                                   # a literal: copied up to its closing quote
            j = i + 1
            while j < n and text[j] != c:
                j += 2 if text[j] == "\\" else 1
            out.append(text[i:j + 1])
            i = j + 1
        elif text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
            out.append(" ")
        else:
            out.append(c)
            i += 1
    lines = [ln.rstrip() for ln in "".join(out).split("\n")]
    return "\n".join(ln for ln in lines if ln)


def source_id() -> str:
    """16 hex digits of SHA-256 over the code the library is built from (csrc/*.hip / *.h / *.cpp and the export map,
    include/torrent_verify.h -- comments stripped -- and the asm generator).  Compiled into the library
    (TV_BUILD_ID=..., read back by _native.build_id()), so a measurement tied to it (profiles/traffic_*.json) applies
    to that build only; a comment edit keeps the id."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h", ".cpp", ".map")))
    for f in [os.path.join(CSRC, f) for f in files] + [os.path.join(ROOT, "include", "torrent_verify.h"),
                                                         os.path.join(ROOT, "tools", "gen_sha1_asm.py")]:
        text = open(f, encoding="utf-8", errors="surrogateescape").read()
        if not f.endswith(".py"):
            text = _code_only(text)
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        h.update(text.encode("utf-8", "surrogateescape"))
    return h.hexdigest()[:16]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    gen = os.path.join(ROOT, "tools", "gen_sha1_asm.py")
    header = os.path.join(CSRC, "sha1_asm.h")
    if force or _newer(header, [gen]):
        subprocess.check_call([sys.executable, gen, "--out", header])
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    host_srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES]
    deps = srcs + host_srcs + [header, os.path.join(CSRC, "tv_internal.h"), os.path.join(CSRC, "tv_host.h"),
                               os.path.join(CSRC, "tv_ctx.h"), os.path.join(CSRC, "tv_options_internal.h"), EXPORTS,
                               os.path.join(CSRC, "tv_plan.h"),
                               os.path.join(ROOT, "include", "torrent_verify.h")]
    if not (force or _newer(LIB, deps)):
        return LIB
    objs = []
    cmds = []
    sid = source_id()
    for s in srcs:
        o = os.path.join(CSRC, os.path.basename(s) + ".o")
        cmds.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                     f"-DTV_SOURCE_ID=\"{sid}\"", "-I", os.path.join(ROOT, "include"), "-c", s, "-o", o])
        objs.append(o)
    procs = []
    for cmd in cmds:                       # (the translation units compile side by side)
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
    bad = [cmd for cmd, p in zip(cmds, procs) if p.wait() != 0]
    if bad:
        raise subprocess.CalledProcessError(1, bad[0])
    for s in host_srcs:
        o = os.path.join(CSRC, os.path.basename(s) + ".o")
        cmd = [CXX, "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        objs.append(o)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", f"-Wl,--version-script={EXPORTS}", "-o", LIB] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
