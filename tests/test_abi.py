"""C ABI checks that need no GPU: the library loads, exports every symbol include/*.h declares,
argument/state errors are reported (not crashed on), and the asm generator's emulator passes."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "torrent_verify.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void)\s+\*?\s*(tv_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol(native):
    lib = native.lib()
    declared = _declared_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(n for n, _, _ in native.SYMBOLS) == declared  # the binding covers the header
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (tv_\w+)", out))
    assert set(declared) <= exported


def test_abi_version_and_no_device_errors(native):
    lib = native.lib()
    assert lib.tv_abi_version() == 1
    n = native.device_count()
    if n == 0:
        with pytest.raises(native.NativeError) as ei:
            native.Context(0)
        assert ei.value.code == native.TV_ERR_ARG and "out of range" in str(ei.value)


def test_cpu_share_equals_the_python_host(native):
    """tv_cpu_share (the TS host's default thread share) reads the CPU share by the rule of
    torrent_amd/_cpu.py cpu_share (cgroup quota, else OMP_NUM_THREADS, else the affinity mask) -- no GPU needed."""
    from torrent_amd import _cpu
    assert native.cpu_share() == _cpu.cpu_share()["cores"]


def test_null_ctx_is_an_error_not_a_crash(native):
    lib = native.lib()
    assert lib.tv_set_layout(None, 1, 1, 1, 0, 1) == native.TV_ERR_ARG
    assert lib.tv_verify(None, None, None) == native.TV_ERR_ARG
    lib.tv_destroy(None)
    buf = bytes(256)
    import ctypes
    b = ctypes.create_string_buffer(256)
    assert lib.tv_last_error(None, b, 256) > 0 and b"NULL" in b.value


def test_asm_generator_emulator():
    """The generated SHA-1 asm instruction streams compute SHA-1 (emulated, vs hashlib)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


@pytest.mark.parametrize("env", [{"TV_GEN_PAIRXOR": "0"}, {"TV_GEN_KROUNDS": "1"}, {"TV_GEN_HPAIR": "1"},
                                 {"TV_GEN_PIPE": "1", "TV_GEN_RING": "20"}, {"TV_GEN_BUFS": "2"},
                                 {"TV_GEN_TWIN_ISSUE": "end"}, {"TV_GEN_TWIN_ISSUE": "spread"},
                                 {"TV_GEN_TWIN_PRE": "0"}, {"TV_GEN_TWIN_WAITS": "0-2-4-6-8", "TV_GEN_TWIN_ISSUE": "end"},
                                 {"TV_GEN_SPLIT_MID": "1", "TV_GEN_RING": "20"}, {"TV_GEN_SPLIT_PRE": "1"}])
def test_asm_generator_emulator_options(env):
    """The generator's A/B options (tools/build_variants.py) still emit streams that compute SHA-1."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--check"],
                       capture_output=True, text=True, env=dict(os.environ, **env))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


@pytest.mark.parametrize("stamp", ["1", "2"])
def test_asm_generator_stamp_headers(tmp_path, stamp):
    """The diagnostic stamp headers (TV_GEN_STAMP, tools/split_stamps.py) still generate: both split loops get the
    accumulator argument(s) and the stamp SGPRs as clobbers; level 2 also brackets the helper's prefetch wait, and its
    LDS-write drain where the helper still drains before the barrier (TV_GEN_HWAIT=0);
    the shipped header's helper waits mid-block (TV_GEN_HWAIT=mid) and the previous form stays available."""
    out = tmp_path / "h.h"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--out", str(out)],
                       capture_output=True, text=True, env=dict(os.environ, TV_GEN_STAMP=stamp))
    assert r.returncode == 0, r.stderr
    h = out.read_text()
    assert f"#define TV_SHA1_STAMP {stamp}" in h
    assert "tv_sha1_rounds_loop(uint32_t h[5], uint32_t addr, uint32_t nsteps, uint32_t& sbar," in h
    assert ('uint32_t& sbar, uint32_t& svm, uint32_t& slg,' in h) == (stamp == "2")
    assert h.count('"s88", "s89", "s90", "s91"') == 4      # split and twin: rounds and helper loops
    assert "tv_sha1_twin_rounds_loop(uint32_t h[5], uint32_t addr, uint32_t nsteps, uint32_t& sbar) {" in h
    assert ("%[svm]" in h) == (stamp == "2") and "%[sbar]" in h
    if stamp == "2":   # the drain stamp needs the drain: the twin helper's, and the split helper's only with the
        # pre-round-4 wait (TV_GEN_HWAIT=0)
        i = h.index("void tv_sha1_helper_loop(")
        assert "%[slg]" not in h[i:h.index("\n}\n", i)] and "%[slg]" in h
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--out", str(out)],
                           capture_output=True, text=True, env=dict(os.environ, TV_GEN_STAMP="2", TV_GEN_HWAIT="0"))
        assert r.returncode == 0 and "%[slg]" in out.read_text(), r.stderr
    shipped = open(os.path.join(ROOT, "torrent_amd", "csrc", "sha1_asm.h")).read()
    assert "TV_SHA1_STAMP" not in shipped and "s_memtime" not in shipped and "s_waitcnt lgkmcnt(10)" in shipped
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--out", str(out)],
                       capture_output=True, text=True, env=dict(os.environ, TV_GEN_HWAIT="0"))
    assert r.returncode == 0 and "s_waitcnt lgkmcnt(10)" not in out.read_text(), r.stderr


def test_generated_header_is_current(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sha1_asm.py"), "--out",
                        str(tmp_path / "h.h")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "h.h").read_text() == open(os.path.join(ROOT, "torrent_amd", "csrc", "sha1_asm.h")).read()


def test_no_oracle_in_product_path():
    """The product package never imports / links / loads the oracle."""
    for dp, _, fs in os.walk(os.path.join(ROOT, "torrent_amd")):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in txt.replace("Oracle", "").lower() or f == "__init__.py", f


def _header_prototypes():
    """(name -> (result C type, [param C types])) for every function include/torrent_verify.h declares."""
    import re
    src = open(os.path.join(ROOT, "include", "torrent_verify.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for m in re.finditer(r"^\s*(void|int)\s+(tv_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.M):
        params = [p.strip() for p in m.group(3).split(",") if p.strip() and p.strip() != "void"]
        types = [re.sub(r"\s*\b\w+$", "", p) if not p.endswith("*") else p for p in params]
        out[m.group(2)] = (m.group(1), [" ".join(t.replace("*", " * ").split()) for t in types])
    return out


def _deno_type(c):
    if "*" in c:
        return "pointer"
    return {"int": "i32", "uint64_t": "u64", "int64_t": "i64", "size_t": "usize", "void": "void"}[c]


def test_deno_and_ctypes_bindings_match_header():
    """ts/verify.ts (the Deno.dlopen table a maintainer adds) and
    torrent_amd/_native.py (its ctypes twin) declare exactly the header's functions with the same
    parameter kinds.  Deno is absent from the image, so this is how the TS binding is checked."""
    import ctypes
    import re
    protos = _header_prototypes()
    assert len(protos) >= 20
    ts = open(os.path.join(ROOT, "ts", "verify.ts")).read()
    table = ts[ts.index("const SYMBOLS = {"):ts.index("} as const;")]
    deno = {}
    for m in re.finditer(r"(tv_\w+):\s*\{\s*parameters:\s*\[([^\]]*)\],\s*result:\s*\"(\w+)\"", table, flags=re.S):
        deno[m.group(1)] = (m.group(3), re.findall(r"\"(\w+)\"", m.group(2)))
    assert set(deno) == set(protos)
    for name, (res, params) in protos.items():
        assert deno[name] == (_deno_type(res), [_deno_type(p) for p in params]), name

    from torrent_amd import _native
    ct = {n: (r, a) for n, r, a in _native.SYMBOLS}
    assert set(ct) == set(protos)
    size = {"int": 4, "uint64_t": 8, "int64_t": 8, "size_t": 8}
    for name, (res, params) in protos.items():
        r, args = ct[name]
        assert (r is None) == (res == "void"), name
        assert len(args) == len(params), name
        for c, a in zip(params, args):
            if "*" in c:
                assert a in (ctypes.c_void_p, ctypes.c_char_p) or hasattr(a, "contents") or a.__name__.startswith("LP_"), (name, c)
            else:
                assert ctypes.sizeof(a) == size[c], (name, c)


def test_product_path_fails_loudly_without_the_library(tmp_path):
    """No CPU fallback: with the HIP library absent, verify_pieces / hash_pieces raise ImportError
    instead of computing anything (a silent fallback would void the parity claims)."""
    code = (
        "from torrent_amd import make_info, verify_pieces, hash_pieces\n"
        "info = make_info(64, bytes(20), 'x', length=64)\n"
        "class S:\n"
        "    def get(self, off, n): return bytes(n)\n"
        "for fn, a in ((verify_pieces, (info, S())), (hash_pieces, (bytes(64), 64))):\n"
        "    try:\n"
        "        fn(*a)\n"
        "    except ImportError as e:\n"
        "        assert 'no CPU fallback' in str(e), e\n"
        "    else:\n"
        "        raise SystemExit(fn.__name__ + ' returned without the library')\n"
        "print('raised')\n")
    env = dict(os.environ, TORRENT_VERIFY_LIB=str(tmp_path / "missing.so"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "raised" in r.stdout, r.stdout + r.stderr


def build_c_consumer(out_dir) -> str:
    """gcc-compile tests/c/abi_consumer.c against include/ and the in-tree library (no Python in
    the consumer: the shape of a Deno FFI / cgo binding)."""
    exe = os.path.join(str(out_dir), "abi_consumer")
    lib_dir = os.path.join(ROOT, "torrent_amd")
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "abi_consumer.c"), "-L", lib_dir, "-ltorrent_verify",
                           f"-Wl,-rpath,{lib_dir}", "-lpthread", "-o", exe])
    return exe


def test_c_consumer_error_paths(native, tmp_path):
    """A plain-C program links the library and gets statuses + messages (never a crash) for NULL
    arguments and, without a GPU, for tv_create."""
    exe = build_c_consumer(tmp_path)
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_buffer_addresses_are_never_copies():
    """_native._addr hands the library the caller's own bytes: a read-only source (a slice of a `bytes`
    payload, as verify_payload stages it) is not duplicated -- a 16 GiB `bytes` payload would otherwise be
    copied whole per shard -- and a read-only output is refused instead of written into a temporary."""
    import ctypes
    import pytest
    from torrent_amd import _native
    b = bytes(range(256)) * 16
    base = ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value
    a, keep = _native._addr(b)
    assert a == base
    a, keep = _native._addr(memoryview(b)[100:900])
    assert a == base + 100 and ctypes.string_at(a, 800) == b[100:900]
    ba = bytearray(b)
    a, keep = _native._addr(memoryview(ba)[7:], writable=True)
    ctypes.memset(a, 0xAB, 1)
    assert ba[7] == 0xAB
    with pytest.raises(TypeError):
        _native._addr(memoryview(b)[1:], writable=True)
    with pytest.raises(TypeError):
        _native._addr(b, writable=True)
    assert _native._addr(None) == (None, None) and _native._addr(bytearray())[0] is None


def _defines(path):
    txt = open(os.path.join(ROOT, path)).read()
    return {m.group(1): int(m.group(2)) for m in
            re.finditer(r"^#define\s+(TV_(?:OPT|COUNTER|ERR|FILE)_\w+)\s+\(?(-?\d+)\)?", txt, re.M)}


def test_option_and_counter_constants_match_header():
    """Every TV_OPT_* / TV_COUNTER_* / TV_ERR_* value of include/torrent_verify.h and of the library's internal
    header (tv_options_internal.h: measurement and test knobs) is the same in the ctypes binding
    (torrent_amd/_native.py), and in every constant ts/verify.ts declares (public ones only)."""
    from torrent_amd import _native
    public = _defines("include/torrent_verify.h")
    internal = _defines("torrent_amd/csrc/tv_options_internal.h")
    assert len(public) >= 25 and len(internal) >= 10
    for name, v in {**public, **internal}.items():
        if name.startswith("TV_FILE_"):
            continue
        assert getattr(_native, name) == v, name
    phases = sorted((v, k) for k, v in internal.items()
                    if k.startswith(("TV_FILE_PHASE_", "TV_FILE_BYTES_", "TV_FILE_ODIRECT_")))
    assert [k.split("_", 3)[3].lower() if k.startswith("TV_FILE_PHASE_") else
            "bytes_" + k.split("_")[-1].lower() if k.startswith("TV_FILE_BYTES_") else
            "odirect_" + k.split("_")[-1].lower() for _, k in phases] == list(_native.TV_FILE_PHASES)
    plan = open(os.path.join(ROOT, "torrent_amd", "csrc", "tv_plan.h")).read()
    assert int(re.search(r"kWinBufsDefault = (\d+);", plan).group(1)) == _native.WIN_BUFS_DEFAULT
    ts = open(os.path.join(ROOT, "ts", "verify.ts")).read()
    for m in re.finditer(r"const\s+(TV_\w+)\s*=\s*(-?\d+)\s*;", ts):
        assert public[m.group(1)] == int(m.group(2)), m.group(1)


def test_public_options_are_what_the_hosts_use():
    """The public header's option set (the reference's whole plugin surface is three methods,
    storage.ts:16-26) is exactly the set the hosts use: ts/verify.ts, the product modules of torrent_amd, and the
    public wrappers of _native.Context.  Measurement and test knobs live in tv_options_internal.h, and no key is in
    both headers."""
    public = {k for k in _defines("include/torrent_verify.h") if k.startswith("TV_OPT_")}
    internal = _defines("torrent_amd/csrc/tv_options_internal.h")
    assert not public & set(internal)
    pub_vals = {v for k, v in _defines("include/torrent_verify.h").items() if k.startswith("TV_OPT_")}
    assert not pub_vals & {v for k, v in internal.items() if k.startswith("TV_OPT_")}
    used = set()
    ts = open(os.path.join(ROOT, "ts", "verify.ts")).read()
    used |= set(re.findall(r"\b(TV_OPT_\w+)\b", ts[ts.index("} as const;"):]))
    pkg = os.path.join(ROOT, "torrent_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py") and f != "_native.py":
            used |= set(re.findall(r"\b(TV_OPT_\w+)\b", open(os.path.join(pkg, f)).read()))
    nat = open(os.path.join(pkg, "_native.py")).read()
    api = nat[nat.index("class Context:"):]
    for m in re.finditer(r"\n    def ([a-z]\w*)\(self[^)]*\)[^:]*:(.*?)(?=\n    def |\Z)", api, re.S):
        used |= set(re.findall(r"\b(TV_OPT_\w+)\b", m.group(2)))
    assert used == public, (sorted(used - public), sorted(public - used))


def test_source_id_ignores_comments_only():
    """The library's build id (torrent_amd/_build.py source_id, compiled in as TV_BUILD_ID) hashes code, not
    comments: a measurement tied to a build (profiles/traffic_*.json) survives a documentation edit, not a code one."""
    from torrent_amd._build import _code_only
    a = 'int f(int x) { // add one\n  return x + 1; /* plain */ }\nconst char* s = "// not a comment";\n'
    b = '/* new header text */\nint f(int x) {\n  return x + 1;   }\n\nconst char* s = "// not a comment";\n'
    assert _code_only(a).split() == _code_only(b).split()
    assert '"// not a comment"' in _code_only(a)
    assert _code_only(a) != _code_only(a.replace("x + 1", "x + 2"))
