"""Host thread budgets across the shards of one call, on CPU: the library's reader / copy
threads (TV_OPT_FILE_THREADS per context) of the concurrently active shards sum to at most the process's CPU
share, in the Python host (torrent_amd/verify.py over torrent_amd/_cpu.py) and in the TS host (ts/verify.ts,
under Node with the JS model of the library).  No GPU: the contexts are recording stand-ins."""
import json
import os

import pytest

from torrent_amd import _cpu, _native, verify
from torrent_amd.metainfo import make_info

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_threads_rule():
    assert _cpu.shard_threads([0] * 8, share=16, node_cpu_count={0: 128}) == [2] * 8
    assert _cpu.shard_threads([0], share=16, node_cpu_count={0: 128}) == [16]
    assert _cpu.shard_threads([0], share=256, node_cpu_count={0: 128}) == [16]           # capped at 16
    assert _cpu.shard_threads([0] * 3, share=2, node_cpu_count={0: 128}) == [1, 1, 1]   # at least one each
    # per NUMA node: four shards on a node with 8 CPUs get 2 each, whatever the process-wide share
    assert _cpu.shard_threads([0, 0, 0, 0, 1, 1, 1, 1], share=64, node_cpu_count={0: 8, 1: 64}) == [2] * 4 + [8] * 4
    assert _cpu.shard_threads([None, None], share=16) == [8, 8]                         # node unknown
    for n in range(1, 17):
        for share in (1, 4, 16, 64, 256):
            t = _cpu.shard_threads([0] * n, share=share, node_cpu_count={0: 256})
            assert sum(t) <= max(share, n) and all(1 <= x <= 16 for x in t)


class _FakeCtx:
    """Records the options a bulk call sets; enough of _native.Context for verify_files / hash_files."""

    def __init__(self, device):
        self.device = device
        self.options = {}
        self.thread_budget = 16

    def set_option(self, key, value):
        self.options[key] = value

    def set_layout(self, *a):
        pass

    def set_digests(self, raw):
        pass

    def counter(self, key):
        assert key == _native.TV_COUNTER_NUMA_NODE
        return 0

    def stage_files(self, paths, fo, lin, lens):
        return [0] * len(paths)

    def verify(self, avail=None):
        return bytes(avail)


@pytest.mark.parametrize("share", [16, 4])
def test_python_host_divides_the_share_among_shards(monkeypatch, share):
    from contextlib import contextmanager
    ctxs = {}

    @contextmanager
    def fake_context(device, slot=0):
        yield ctxs.setdefault((device, slot), _FakeCtx(device))

    monkeypatch.setattr(verify, "_context", fake_context)
    monkeypatch.setattr(verify, "_node_of", {})
    monkeypatch.setattr(_cpu, "cpu_share", lambda: {"cores": share})
    monkeypatch.setattr(_cpu, "node_cpus", lambda node: 128)
    L, P = 1 << 20, 256
    info = make_info(L, bytes(20 * P), "t.bin", length=L * P)
    verify.verify_files(info, "/nonexistent/budget", devices=[0] * 8)
    threads = [c.options[_native.TV_OPT_FILE_THREADS] for c in ctxs.values()]
    assert len(threads) == 8 and sum(threads) <= max(share, 8) and min(threads) >= 1   # (one each at least)
    # one device: the whole share (up to 16)
    ctxs.clear()
    verify.verify_files(info, "/nonexistent/budget", devices=[0])
    assert [c.options[_native.TV_OPT_FILE_THREADS] for c in ctxs.values()] == [min(16, share)]


@pytest.mark.skipif(not __import__("shutil").which("node"), reason="needs node")
def test_ts_host_divides_the_share_among_shards(tmp_path):
    from tests.test_ts_binding import HARNESS, _info_json, erased_module, run_node
    mod = erased_module(tmp_path)
    L, P = 1 << 16, 512
    (tmp_path / "spec.json").write_text(json.dumps(_info_json(L, L * P, bytes(20 * P))))
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
Deno.fakeAvailOnly = true;
globalThis.navigator = {{ hardwareConcurrency: 16 }};
const fs = require("fs");
import("{mod}").then(async (m) => {{
  const d = JSON.parse(fs.readFileSync("{tmp_path}/spec.json", "utf8"));
  const raw = Buffer.from(d.pieces, "base64");
  const pieces = [];
  for (let i = 0; i < raw.length; i += 20) pieces.push(new Uint8Array(raw.subarray(i, i + 20)));
  const info = {{ pieceLength: d.pieceLength, length: d.length, pieces, name: d.name, private: 0 }};
  const res = {{}};
  for (const [name, opts] of [["8 devices", {{ devices: Array(8).fill(0) }}], ["1 device", {{}}],
                              ["8 devices, threads 4", {{ devices: Array(8).fill(0), threads: 4 }}]]) {{
    await m.releaseContexts();
    Deno.fakeReset();
    await m.verifyFiles(info, "/nonexistent/budget", opts);
    res[name] = [...Deno.fakeContexts.values()].map((c) => (c.options || {{}})[8]);
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    assert res["8 devices"] == [2] * 8
    assert res["1 device"] == [16]
    assert res["8 devices, threads 4"] == [1] * 8


def test_storage_paths_honour_an_explicit_thread_count():
    """verify_pieces / verify_stream: the default (threads=None) is _STORAGE_THREADS capped at the
    shard's CPU part; an explicit count -- e.g. 32 readers for a Storage whose gets mostly wait -- is used as given."""
    ctx = _FakeCtx(0)
    ctx.thread_budget = 2
    assert verify._storage_threads(ctx, None) == 2
    ctx.thread_budget = 16
    assert verify._storage_threads(ctx, None) == verify._STORAGE_THREADS
    assert verify._storage_threads(ctx, 32) == 32
    assert verify._storage_threads(ctx, 1) == 1
    assert verify._storage_threads(ctx, 0) == 1


def test_stream_rule_is_the_same_in_both_hosts(tmp_path):
    """verify_files / verifyFiles choose streamed columns over windows by the same rule (torrent_amd/verify.py
    _stream_wins, ts/verify.ts streamWins); both hand the budget to the library, which sizes the columns."""
    import shutil
    cases = [(1 << 20, 16384, None), (1 << 20, 16384, 1 << 29), (1 << 20, 16384, 1 << 30), (1 << 20, 16384, 2 << 30),
             (4 << 20, 51200, 3 << 30), (4 << 20, 51200, 4 << 30), (256 << 10, 100, 1 << 20), (1000, 37, 5000),
             (65536, 1000, 1), (1 << 20, 10, 1 << 29)]
    want = [verify._stream_wins(L, n, b) for L, n, b in cases]
    assert want[1] and not want[2] and not want[0] and want[6] and not want[9]
    if not shutil.which("node"):
        pytest.skip("needs node")
    from tests.test_ts_binding import erased_module, run_node
    mod = erased_module(tmp_path)
    out = run_node(tmp_path, f"""
import("{mod}").then((m) => {{
  const cases = {json.dumps([[L, n, b] for L, n, b in cases])};
  console.log(JSON.stringify(cases.map(([L, n, b]) => m.streamWins(L, n, b === null ? undefined : b))));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    assert json.loads(out) == want


def test_payload_streams_exactly_when_the_shard_exceeds_the_budget():
    """verify_payload streams (tv_verify_host, windows x columns) by default exactly when the shard's padded payload
    -- tv_set_layout's count x (L rounded up to 64 + 256) + 256 bytes -- exceeds the budget; without a budget the
    library's own (free HBM) decides and the shard is held resident.  _stream_wins (verify_files) is a subset."""
    L, n = 1 << 20, 16384
    need = n * (L + 256) + 256
    assert not verify._exceeds(L, n, None) and not verify._exceeds(L, n, 0)
    assert not verify._exceeds(L, n, need) and verify._exceeds(L, n, need - 1)
    assert verify._exceeds(1000, 37, 37 * (1024 + 256))               # (1000 rounds up to 1024)
    assert not verify._exceeds(1000, 37, 37 * (1024 + 256) + 256)
    for b in (1 << 28, 1 << 29, 1 << 30, 2 << 30, need - 1, need):
        assert not verify._stream_wins(L, n, b) or verify._exceeds(L, n, b)
