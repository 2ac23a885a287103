"""Build A/B variants of libtorrent_verify.so from generator settings (tools/gen_sha1_asm.py TV_GEN_*).

    python tools/build_variants.py name:KEY=VAL,KEY=VAL [name2:...]
e.g.  python tools/build_variants.py base:BUFS=2,PIPE=0,RING=16 pipe:BUFS=3,PIPE=1,RING=20
A key D_<MACRO> is passed to hipcc as -D<MACRO>=VAL instead (e.g. lane3:D_TV_LANE_DEPTH=3).

Each variant's header is generated into torrent_amd/csrc/sha1_asm.h, the library is linked to
build/variants/libtv_<name>.so, and the shipped header is regenerated at the end.  Load a variant with
TORRENT_VERIFY_LIB=build/variants/libtv_<name>.so (tools/variant_bench.py does)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "torrent_amd", "csrc")
OUT = os.path.join(ROOT, "build", "variants")
HIPCC = "/opt/rocm/bin/hipcc"


def build(name, env):
    e = dict(os.environ)
    e.update({f"TV_GEN_{k}": v for k, v in env.items() if not k.startswith("D_")})
    defs = [f"-D{k[2:]}={v}" for k, v in env.items() if k.startswith("D_")]
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--out",
                           os.path.join(CSRC, "sha1_asm.h")], env=e, stdout=subprocess.DEVNULL)
    os.makedirs(OUT, exist_ok=True)
    objs = []
    from torrent_amd._build import SOURCES, EXPORTS
    for src in SOURCES:
        o = os.path.join(OUT, f"{name}_{src}.o")
        subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I",
                               os.path.join(ROOT, "include")] + defs + ["-c", os.path.join(CSRC, src), "-o", o])
        objs.append(o)
    o = os.path.join(OUT, f"{name}_tv_host.o")
    subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, "tv_host.cpp"), "-o", o])
    objs.append(o)
    lib = os.path.join(OUT, f"libtv_{name}.so")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", f"-Wl,--version-script={EXPORTS}", "-o", lib] + objs)
    for x in objs:
        os.remove(x)
    print(lib)


def main():
    try:
        for spec in sys.argv[1:]:
            name, _, kv = spec.partition(":")
            build(name, dict(x.split("=") for x in kv.split(",") if x))
    finally:
        subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--out",
                               os.path.join(CSRC, "sha1_asm.h")], stdout=subprocess.DEVNULL)


if __name__ == "__main__":
    main()
