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
