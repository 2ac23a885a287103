"""ts/verify.ts, executed: the Deno binding run under Node 12 with a Deno FFI shim (tests/ts_harness).

Deno is absent from the image, so the binding a maintainer would add to the reference is type-erased
(tests/ts_harness/erase_ts.py: annotations, interfaces, casts, generics, modifiers only) and run by Node 12
with `Deno.dlopen` / `Deno.UnsafePointer` / `Deno.UnsafePointerView` provided by a small N-API addon
(tests/ts_harness/deno_ffi.cc) that calls the real libtorrent_verify.so (`nonblocking` symbols on libuv worker
threads, as Deno runs them on its blocking pool, so shards' calls overlap).  On CPU: the erased module parses,
its pure helpers equal the Python host's, and the whole symbol table binds through the shim.  On the GPU
(`-m gpu`): verifyPieces, verifyStream, verifyFiles (zero-length segments in a directory's place and in a
missing directory), verifyPiece, hashPieces and the PieceVerifier flush policy (the count bound, and the
age timer alone) return the reference's bits,
computed here with the Python mirror and hashlib as the checker -- the same inputs the Python host is
tested on, so the two hosts cannot drift apart unseen.
"""
import base64
import hashlib
import json
import os
import random
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "ts_harness")
ADDON = os.path.join(HARNESS, "deno_ffi.node")
LIB = os.path.join(ROOT, "torrent_amd", "libtorrent_verify.so")
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="needs node")


def build_addon() -> str:
    """Compile the N-API Deno FFI shim (test infrastructure; __graft_entry__.build() also builds it)."""
    src = os.path.join(HARNESS, "deno_ffi.cc")
    if not os.path.exists(ADDON) or os.path.getmtime(ADDON) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-DNODE_GYP_MODULE_NAME=deno_ffi",
                               "-I/usr/include/node", src, "-o", ADDON])
    return ADDON


WALK = os.path.join(HARNESS, "walk_main")


def build_walk() -> str:
    """The library's file-table walk (tv_plan.h walk_file_table) as a CPU program (tests/c/walk_main.cpp): the JS
    model of the library runs it for tv_stage_file_table, so the CPU tests see the library's own walk."""
    src = os.path.join(ROOT, "tests", "c", "walk_main.cpp")
    hdr = os.path.join(ROOT, "torrent_amd", "csrc", "tv_plan.h")
    if not os.path.exists(WALK) or os.path.getmtime(WALK) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", src, "-o", WALK])
    return WALK


def erased_module(tmp_path) -> str:
    import sys
    sys.path.insert(0, HARNESS)
    from erase_ts import erase
    out = os.path.join(str(tmp_path), "verify.mjs")
    with open(out, "w") as f:
        f.write(erase(open(os.path.join(ROOT, "ts", "verify.ts")).read()))
    return out


def run_node(tmp_path, script: str) -> str:
    path = os.path.join(str(tmp_path), "probe.mjs")
    with open(path, "w") as f:
        f.write(script)
    env = dict(os.environ, TV_WALK_EXE=build_walk())
    r = subprocess.run([NODE, path], capture_output=True, text=True, timeout=120, cwd=HARNESS, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_erased_binding_parses_and_helpers_match(tmp_path):
    """The erased module is valid Node 12 JavaScript; shardRanges and flushCostMs equal the Python host's."""
    from torrent_amd.incremental import flush_cost_ms
    from torrent_amd.verify import shard_ranges
    mod = erased_module(tmp_path)
    r = subprocess.run([NODE, "--check", mod], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    build_addon()
    cases = [(0, 1), (1, 1), (7, 3), (203, 8), (51200, 8), (16384, 3), (100, 16)]
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
require("./deno_shim.js");
import("{mod}").then((m) => {{
  const cases = {json.dumps(cases)};
  console.log(JSON.stringify({{ shards: cases.map(([p, n]) => m.shardRanges(p, n)),
                               costs: [16384, 262144, 1048576, 4194304].map((L) => m.flushCostMs(L)) }}));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    got = json.loads(out)
    assert got["shards"] == [[list(x) for x in shard_ranges(p, n)] for p, n in cases]
    for L, c in zip([16384, 262144, 1048576, 4194304], got["costs"]):
        assert abs(c - flush_cost_ms(L)) < 1e-9


def test_symbol_table_binds_through_the_shim(tmp_path):
    """Deno.dlopen of the binding's whole SYMBOLS table on the real library (every symbol resolves, the ABI
    version check passes): a zero-piece verifyPieces loads the library and returns an empty bitfield without
    touching a device."""
    mod = erased_module(tmp_path)
    build_addon()
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
require("./deno_shim.js");
import("{mod}").then(async (m) => {{
  const info = {{ pieceLength: 16384, length: 0, pieces: [], name: "t", private: 0 }};
  const bf = await m.verifyPieces(info, {{ async get() {{ return null; }} }}, {{ libPath: "{LIB}" }});
  console.log(JSON.stringify({{ n: bf.length }}));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    assert json.loads(out) == {"n": 0}


# ------------------------------------------------------------------------------------------------ GPU

def _b64(b) -> str:
    return base64.b64encode(bytes(b)).decode()


def _info_json(L, total, digests, files=None, name="t.bin"):
    d = {"pieceLength": L, "length": total, "pieces": _b64(digests), "name": name}
    if files is not None:
        d["files"] = [{"length": n, "path": list(p)} for n, p in files]
    return d


def _expect_linear(payload, L, digests, unreadable=()):
    total = len(payload)
    P = len(digests) // 20 + (1 if len(digests) % 20 else 0)
    bits = bytearray((P + 7) // 8)
    for i in range(P):
        n = (total % L) if (i == P - 1 and total % L) else L
        d = digests[20 * i:20 * i + 20]
        if i in unreadable or i * L + n > total or len(d) != 20:
            continue
        if hashlib.sha1(payload[i * L:i * L + n]).digest() == d:
            bits[i >> 3] |= 0x80 >> (i & 7)
    return bits.hex()


@pytest.mark.gpu
def test_ts_binding_on_the_gpu(native, tmp_path, monkeypatch):
    from torrent_amd.metainfo import FileInfo, make_info
    from torrent_amd.piece import BLOCK_SIZE, piece_length
    from torrent_amd.storage import Storage, fs_storage
    mod = erased_module(tmp_path)
    build_addon()
    rng = random.Random(7)
    cases, expect = [], {}

    # verifyPieces / verifyStream over in-memory storage: short last piece, corrupted data, unreadable pieces,
    # a ragged digest string; one and three shards; streamed with a narrow column (several per piece)
    for k, (L, P, last) in enumerate([(16384, 61, 999), (65536 + 64, 40, 65536 + 64), (262144, 9, 5)]):
        total = L * (P - 1) + last
        payload = bytearray(rng.getrandbits(8) for _ in range(total))
        digests = bytearray(b"".join(hashlib.sha1(bytes(payload[i * L:(i + 1) * L])).digest() for i in range(P)))
        for i in rng.sample(range(P), 3):
            payload[i * L] ^= 0x40
        if k == 2:
            digests = digests[:-7]
        unreadable = sorted(rng.sample(range(P), 2))
        for devices in ([0], [0, 0, 0]):
            for kind in ("pieces", "stream"):
                name = f"{kind}{k}_{len(devices)}"
                cases.append({"name": name, "kind": kind, "info": _info_json(L, total, digests), "devices": devices,
                              "payload": _b64(payload), "unreadable": unreadable, "chunk": 4096 if k == 1 else 0})
                expect[name] = _expect_linear(bytes(payload), L, bytes(digests), set(unreadable))
        # a row of the wrong length makes its piece unreadable (verifyStream)
        name = f"stream_wrong{k}"
        cases.append({"name": name, "kind": "stream", "info": _info_json(L, total, digests), "devices": [0],
                      "payload": _b64(payload), "unreadable": [], "wrongLength": [1]})
        expect[name] = _expect_linear(bytes(payload), L, bytes(digests), {1})

    # verifyFiles on disk: a directory and a missing directory in zero-length files' places, a missing file,
    # a short file; expected bits from Storage(fs_storage).get on a copy (that get creates files)
    L = 4096
    names = [("a",), ("z_dir",), ("b",), ("nodir", "z"), ("c",), ("z_missing",), ("d",), ("gone",), ("e",), ("short",)]
    sizes = [3 * L, 0, 2 * L + 100, 0, L - 100, 0, 2 * L, 700, L + 7, 3000]
    payload = bytes(rng.getrandbits(8) for _ in range(sum(sizes)))
    P = -(-len(payload) // L)
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    files = list(zip(sizes, names))
    for root in ("dl", "ref"):
        off = 0
        for n, p in files:
            q = tmp_path.joinpath(root, *p)
            if p == ("z_dir",):
                q.mkdir(parents=True, exist_ok=True)
            elif p not in (("nodir", "z"), ("z_missing",), ("gone",)):
                q.parent.mkdir(parents=True, exist_ok=True)
                q.write_bytes(payload[off:off + (n - 1 if p == ("short",) else n)])
            off += n
    monkeypatch.chdir(tmp_path)
    info = make_info(L, digests, "t", files=[FileInfo(n, list(p)) for n, p in files])
    ref = Storage(fs_storage, info, str(tmp_path / "ref"))
    bits = bytearray((P + 7) // 8)
    for i in range(P):
        got = ref.get(i * L, piece_length(i, info))
        if got is not None and hashlib.sha1(bytes(got)).digest() == digests[20 * i:20 * i + 20]:
            bits[i >> 3] |= 0x80 >> (i & 7)
    assert 0 < sum(bin(x).count("1") for x in bits) < P
    before = sorted(str(x) for x in (tmp_path / "dl").rglob("*"))
    for devices in ([0], [0, 0]):
        name = f"files_{len(devices)}"
        cases.append({"name": name, "kind": "files", "info": _info_json(L, len(payload), digests, files, "t"),
                      "dir": str(tmp_path / "dl"), "devices": devices})
        expect[name] = bits.hex()
        # the streamed form (tv_stream_file_table): columns sized to a budget of a few pieces
        name = f"files_streamed_{len(devices)}"
        cases.append({"name": name, "kind": "files", "info": _info_json(L, len(payload), digests, files, "t"),
                      "dir": str(tmp_path / "dl"), "devices": devices, "stream": True, "budget": 3 * (L + 512)})
        expect[name] = bits.hex()

    # the streamed form on 5,000 pieces: windows of 2,048 pieces x two 512-byte columns within the budget (the
    # library's geometry), a short last piece, files ending mid-piece, two corrupted pieces at window edges
    L, P = 1024, 5000
    total = L * (P - 1) + 333
    payload = bytearray(rng.randbytes(total))
    digests = b"".join(hashlib.sha1(bytes(payload[i * L:(i + 1) * L])).digest() for i in range(P))
    for i in (2047, 4096):
        payload[i * L + 5] ^= 0x01
    sizes = [1500 * L + 77, 2600 * L - 77, total - 4100 * L]
    files = [(n, (f"w{k}.bin",)) for k, n in enumerate(sizes)]
    off = 0
    for n, p in files:
        q = tmp_path.joinpath("dl2", *p)
        q.parent.mkdir(parents=True, exist_ok=True)
        q.write_bytes(bytes(payload[off:off + n]))
        off += n
    bits = bytearray((P + 7) // 8)
    for i in range(P):
        if i not in (2047, 4096):
            bits[i >> 3] |= 0x80 >> (i & 7)
    for devices in ([0], [0, 0]):
        name = f"files_streamed_windows_{len(devices)}"
        cases.append({"name": name, "kind": "files", "info": _info_json(L, total, digests, files, "t"),
                      "dir": str(tmp_path / "dl2"), "devices": devices, "stream": True,
                      "budget": 2 * (2048 * (512 + 256) + 256)})
        expect[name] = bits.hex()

    # verifyPiece and hashPieces
    L = 262144
    blob = bytes(rng.getrandbits(8) for _ in range(3 * L + 12345))
    digests = b"".join(hashlib.sha1(blob[i * L:(i + 1) * L]).digest() for i in range(4))
    for i, data, want in [(0, blob[:L], True), (3, blob[3 * L:], True), (1, blob[L:2 * L - 1] + b"x", False),
                          (2, blob[2 * L:3 * L - 1], False)]:
        cases.append({"name": f"piece{i}", "kind": "piece", "info": _info_json(L, len(blob), digests),
                      "index": i, "bytes": _b64(data)})
        expect[f"piece{i}"] = want
    cases.append({"name": "hash", "kind": "hash", "payload": _b64(blob), "pieceLength": L})
    expect["hash"] = digests.hex()
    # hashPieces sharded over three contexts (21 pieces: shards of 8, 8 and 5, the last one short)
    L2 = 16384
    blob2 = bytes(rng.getrandbits(8) for _ in range(20 * L2 + 999))
    cases.append({"name": "hash3", "kind": "hash", "payload": _b64(blob2), "pieceLength": L2, "devices": [0, 0, 0]})
    expect["hash3"] = b"".join(hashlib.sha1(blob2[i * L2:(i + 1) * L2]).digest() for i in range(21)).hex()

    # PieceVerifier: blocks in random order, one corrupted, automatic flushes at 8 pending pieces
    L, P = 2 * BLOCK_SIZE, 37
    total = L * (P - 1) + BLOCK_SIZE + 100
    payload = bytes(rng.getrandbits(8) for _ in range(total))
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    blocks = []
    for i in range(P):
        n = L if i < P - 1 else total - (P - 1) * L
        blocks += [[i, o, payload[i * L + o:i * L + min(n, o + BLOCK_SIZE)]] for o in range(0, n, BLOCK_SIZE)]
    rng.shuffle(blocks)
    bad = blocks[5][0]
    blocks[5][2] = bytes(b ^ 1 for b in blocks[5][2])
    cases.append({"name": "verifier", "kind": "verifier", "info": _info_json(L, total, digests),
                  "flushPieces": 8, "flushAgeMs": None, "blocks": [[i, o, _b64(d)] for i, o, d in blocks]})
    # the age bound only: the timer flushes what is pending while no block arrives
    cases.append({"name": "verifier_age", "kind": "verifier", "info": _info_json(L, total, digests),
                  "flushPieces": None, "flushAgeMs": 2, "settleMs": 200,
                  "blocks": [[i, o, _b64(d)] for i, o, d in blocks]})

    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"lib": LIB, "cases": cases}))
    out = tmp_path / "out.json"
    r = subprocess.run([NODE, os.path.join(HARNESS, "run_verify_ts.mjs"), mod, str(spec), str(out)],
                       capture_output=True, text=True, timeout=600, cwd=HARNESS)
    assert r.returncode == 0, r.stdout + r.stderr
    res = {x["name"]: x for x in json.loads(out.read_text())}
    for name, want in expect.items():
        got = res[name]
        assert "error" not in got, (name, got.get("error"))
        key = {"piece": "ok", "hash": "pieces"}.get(got["kind"], "bitfield")
        assert got[key] == want, (name, got[key], want)
    assert sorted(str(x) for x in (tmp_path / "dl").rglob("*")) == before        # verifyFiles created nothing
    v = res["verifier"]
    assert "error" not in v, v.get("error")
    results = {i: ok for i, ok in v["auto"] + v["final"]}
    assert results == {i: i != bad for i in range(P)}
    assert v["autoFlushes"] == len(v["auto"]) // 8 and len(v["auto"]) == 8 * (P // 8)
    want_bits = bytearray((P + 7) // 8)
    for i in range(P):
        if i != bad:
            want_bits[i >> 3] |= 0x80 >> (i & 7)
    assert v["bitfield"] == want_bits.hex()
    va = res["verifier_age"]
    assert "error" not in va, va.get("error")
    assert {i: ok for i, ok in va["auto"] + va["final"]} == {i: i != bad for i in range(P)}
    assert va["autoFlushes"] >= 1 and va["final"] == [] and va["bitfield"] == want_bits.hex()


def test_piece_verifier_policy_on_cpu(tmp_path):
    """PieceVerifier's flush policy on CPU against a JavaScript model of the library (tests/ts_harness/
    fake_deno.js: node's SHA-1 as the checker, nonblocking calls resolving on a later turn of the event loop):
    the count bound flushes every K completed pieces; the age bound alone, through its timer, delivers every
    result within the settle time even when the timer fires before the oldest piece is T ms old (timers are
    millisecond-granular), over 40 trials with bursts and idle gaps; a corrupted block re-sent intact
    verifies."""
    mod = erased_module(tmp_path)
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const crypto = require("crypto");
const sleep = (ms) => new Promise((r) => setTimeout(r, ms));
import("{mod}").then(async (m) => {{
  const L = 32768, P = 29, total = L * (P - 1) + 1000;
  const payload = crypto.randomBytes(total);
  const pieces = [];
  for (let i = 0; i < P; i++) pieces.push(crypto.createHash("sha1").update(payload.slice(i * L, (i + 1) * L)).digest());
  const info = {{ pieceLength: L, length: total, pieces, name: "t", private: 0 }};
  const blocks = [];
  for (let i = 0; i < P; i++) {{
    const n = i === P - 1 ? 1000 : L;
    for (let o = 0; o < n; o += 16384) blocks.push([i, o, payload.slice(i * L + o, i * L + Math.min(n, o + 16384))]);
  }}
  const res = {{ count: null, age: [] }};
  // count bound
  {{
    const got = [];
    const pv = new m.PieceVerifier(info, {{ flushPieces: 4, flushAgeMs: null, onVerified: (i, ok) => got.push([i, ok]) }});
    for (const [i, o, b] of blocks) await pv.onBlock(i, o, b);
    const fin = await pv.flush();
    res.count = {{ auto: got.length, autoFlushes: pv.autoFlushes, final: fin.length,
                   all: [...got, ...fin].filter(([, ok]) => ok).length }};
    await pv.close();
  }}
  // age bound only, bursts and gaps
  for (let trial = 0; trial < 40; trial++) {{
    const got = [];
    const pv = new m.PieceVerifier(info, {{ flushPieces: null, flushAgeMs: 2, onVerified: (i, ok) => got.push([i, ok]) }});
    const order = blocks.slice().sort(() => Math.random() - 0.5);
    let k = 0;
    for (const [i, o, b] of order) {{
      await pv.onBlock(i, o, i === 3 && o === 0 && trial % 2 ? Buffer.alloc(b.length) : b);
      if (++k % (3 + trial % 5) === 0) await sleep(trial % 3);
    }}
    if (trial % 2) {{                                 // once the corrupted piece failed: both blocks re-sent
      await sleep(10);                                 // (re-sends of a piece still pending are ignored)
      for (const o of [0, 16384]) await pv.onBlock(3, o, payload.slice(3 * L + o, 3 * L + o + 16384));
    }}
    await sleep(60);
    const fin = await pv.flush();
    const have = Array.from({{ length: P }}, (_, i) => (pv.bitfield[i >> 3] >> (7 - (i % 8))) & 1);
    res.age.push({{ auto: got.length, final: fin.length, autoFlushes: pv.autoFlushes, have: have.join("") }});
    await pv.close();
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    P = 29
    assert res["count"] == {"auto": 28, "autoFlushes": 7, "final": 1, "all": P}
    for t, r in enumerate(res["age"]):
        assert r["final"] == 0, (t, r)                     # the timer delivered everything
        assert r["autoFlushes"] >= 1 and r["have"] == "1" * P, (t, r)


class _PlanCtx:
    """Records what verify._files_shard hands the library (the Python host's plan)."""

    def __init__(self):
        self.segments = []

    def set_option(self, key, value):
        pass

    def stage_files(self, paths, fo, lin, lens):
        # (Storage keeps the directory relative to the working directory, storage.ts; compare absolute paths)
        self.segments += [[os.path.abspath(p), int(a), int(b), int(c)] for p, a, b, c in zip(paths, fo, lin, lens)]
        return [0] * len(paths)


def test_verify_files_plan_equals_the_python_host(tmp_path):
    """verifyFiles (ts/verify.ts) and verify_files (torrent_amd/verify.py) walk the file table on their own;
    for the 48 seeded random layouts of tests/test_gpu_fuzz.py, on 1 and 3 shards, both hand the library the
    same segments (path, file offset, linear offset, length; zero-length ones included) and the same
    availability bits -- checked on CPU with the JS model of the library recording the TS plan."""
    from tests.test_gpu_fuzz import SEEDS, _draw
    from torrent_amd import verify
    from torrent_amd.storage import Storage, fs_storage
    mod = erased_module(tmp_path)
    d = "/nonexistent/plan/dl"
    spec, want = [], []
    for seed in SEEDS:
        info = _draw(seed)[0]
        spec.append(_info_json(info.piece_length, info.length, info.pieces_raw,
                               None if info.files is None else [(f.length, f.path) for f in info.files],
                               info.name))
        st = Storage(fs_storage, info, d)
        per_n = {}
        for n in (1, 3):
            shards, bits = {}, []
            for first, count in verify.shard_ranges(info.n_pieces, n):
                if not count:
                    continue
                ctx = _PlanCtx()
                avail = verify._files_shard(ctx, info, st, first, count, threads=1)
                shards[str(first)] = sorted(ctx.segments)
                bits += [(avail[j >> 3] >> (7 - (j & 7))) & 1 for j in range(count)]
            per_n[str(n)] = {"shards": shards, "bits": "".join(map(str, bits))}
        want.append(per_n)
    (tmp_path / "spec.json").write_text(json.dumps(spec))
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
Deno.fakeAvailOnly = true;
const fs = require("fs");
import("{mod}").then(async (m) => {{
  const spec = JSON.parse(fs.readFileSync("{tmp_path}/spec.json", "utf8"));
  const res = [];
  for (const d of spec) {{
    const raw = Buffer.from(d.pieces, "base64");
    const pieces = [];
    for (let i = 0; i < raw.length; i += 20) pieces.push(new Uint8Array(raw.subarray(i, Math.min(raw.length, i + 20))));
    const info = {{ pieceLength: d.pieceLength, length: d.length, pieces, name: d.name, private: 0 }};
    if (d.files) info.files = d.files;
    const per = {{}};
    for (const n of [1, 3]) {{
      await m.releaseContexts();
      Deno.fakeReset();
      const bf = await m.verifyFiles(info, "{d}", {{ devices: Array(n).fill(0) }});
      const shards = {{}};
      for (const c of Deno.fakeContexts.values()) {{
        if (c.segments) shards[String(c.first)] = c.segments.slice().sort((x, y) =>
          x[0] < y[0] ? -1 : x[0] > y[0] ? 1 : x[1] - y[1] || x[2] - y[2] || x[3] - y[3]);
      }}
      let bits = "";
      for (let i = 0; i < pieces.length; i++) bits += (bf[i >> 3] >> (7 - (i % 8))) & 1;
      per[String(n)] = {{ shards, bits }};
    }}
    res.push(per);
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    got = json.loads(out)
    for seed, g, w in zip(SEEDS, got, want):
        for n in ("1", "3"):
            g[n]["shards"] = {k: sorted([os.path.abspath(x[0])] + x[1:] for x in v) for k, v in g[n]["shards"].items()}
            assert g[n]["bits"] == w[n]["bits"], (seed, n)
            ws = {k: v for k, v in w[n]["shards"].items() if v}
            assert g[n]["shards"] == ws, (seed, n)


def test_verify_files_paths_in_one_buffer(tmp_path):
    """verifyFiles hands the library every path from ONE NUL-separated buffer (interior pointers): non-ASCII names
    (2-, 3- and 4-byte UTF-8, a surrogate pair among them) arrive intact and in order, and a name holding a NUL --
    which Deno.open refuses, so fsStorage.get's piece is null -- arrives as "", which the library cannot open
    either.  CPU, with the JS model of the library recording the plan."""
    mod = erased_module(tmp_path)
    L = 4096
    names = [["a", "caf\u00e9.bin"], ["\u65e5\u672c", "x.bin"], ["e\U0001f600.bin"], ["bad\u0000name"], ["z.bin"]]
    sizes = [3000, 5000, 0, 700, 4000]
    total = sum(sizes)
    P = -(-total // L)
    spec = _info_json(L, total, bytes(20 * P), list(zip(sizes, names)), "t")
    (tmp_path / "spec.json").write_text(json.dumps(spec))
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
Deno.fakeAvailOnly = true;
const fs = require("fs");
import("{mod}").then(async (m) => {{
  const d = JSON.parse(fs.readFileSync("{tmp_path}/spec.json", "utf8"));
  const info = {{ pieceLength: d.pieceLength, length: d.length, pieces: [], name: d.name, private: 0, files: d.files }};
  const raw = Buffer.from(d.pieces, "base64");
  for (let i = 0; i < raw.length; i += 20) info.pieces.push(new Uint8Array(raw.subarray(i, i + 20)));
  await m.verifyFiles(info, "/r");
  const segs = [];
  for (const c of Deno.fakeContexts.values()) if (c.segments) segs.push(...c.segments);
  console.log(JSON.stringify(segs));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    segs = json.loads(out)
    want = [("/r/" + "/".join(p) if "\0" not in "".join(p) else "") for p in names]
    got_paths = [sg[0] for sg in segs]
    assert set(got_paths) <= set(want), got_paths
    for k, (n, p) in enumerate(zip(sizes, names)):
        if n:
            assert any(sg[0] == want[k] and sg[3] > 0 for sg in segs), (k, got_paths)
    assert "" in got_paths                                          # the NUL name: unopenable, as in Deno
    # the Python host hands the library the same paths ("" for the NUL name; no exception)
    from torrent_amd import make_info, verify
    from torrent_amd.metainfo import FileInfo
    from torrent_amd.storage import Storage, fs_storage

    class Raw(_PlanCtx):
        def stage_files(self, paths, fo, lin, lens):
            # (Storage keeps the directory relative to the working directory, storage.ts: compare absolute paths)
            self.segments += [os.path.abspath(p) if p else "" for p, n in zip(paths, lens) if n]
            return [0] * len(paths)

    info = make_info(L, bytes(20 * P), "t", files=[FileInfo(n, p) for n, p in zip(sizes, names)])
    ctx = Raw()
    verify._files_shard(ctx, info, Storage(fs_storage, info, "/r"), 0, P, threads=1)
    assert sorted(set(ctx.segments)) == sorted({sg[0] for sg in segs if sg[3] > 0})


def test_verify_stream_host_logic_on_cpu(tmp_path):
    """verifyStream's host side (ts/verify.ts: request loop, row lengths, unreadable rows, the worker pool of
    reads, shard concatenation) on CPU against the JS model of the tv_stream_* protocol (several requests per
    column; column widths L, 64 B and 4 KiB) for the 48 seeded fuzz layouts on 1 and 3 shards, with
    unreadable pieces and rows one byte too long: the bits equal hashlib over Storage.get's bytes."""
    from tests.test_gpu_fuzz import SEEDS, _draw
    from torrent_amd.piece import piece_length
    import random as _random
    mod = erased_module(tmp_path)
    spec, want = [], []
    for seed in SEEDS:
        info, payload = _draw(seed)[:2]
        P, L, total = info.n_pieces, info.piece_length, info.length
        rng = _random.Random(seed)
        unreadable = sorted(rng.sample(range(P), min(2, P)))
        wrong = sorted(rng.sample(range(P), 1))
        spec.append({"info": _info_json(L, total, info.pieces_raw), "payload": _b64(payload[:total]),
                     "unreadable": unreadable, "wrong": wrong, "chunk": rng.choice([0, 64, 4096])})
        bits = ""
        for i in range(P):
            n = piece_length(i, info)
            d = info.pieces_raw[20 * i:20 * i + 20]
            ok = (i not in unreadable and i not in wrong and i * L + n <= total and len(d) == 20 and
                  hashlib.sha1(payload[i * L:i * L + n]).digest() == d)
            bits += "1" if ok else "0"
        want.append(bits)
    (tmp_path / "spec.json").write_text(json.dumps(spec))
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const fs = require("fs");
import("{mod}").then(async (m) => {{
  const spec = JSON.parse(fs.readFileSync("{tmp_path}/spec.json", "utf8"));
  const res = [];
  for (const d of spec) {{
    const raw = Buffer.from(d.info.pieces, "base64");
    const pieces = [];
    for (let i = 0; i < raw.length; i += 20) pieces.push(new Uint8Array(raw.subarray(i, Math.min(raw.length, i + 20))));
    const info = {{ pieceLength: d.info.pieceLength, length: d.info.length, pieces, name: "t", private: 0 }};
    const payload = new Uint8Array(Buffer.from(d.payload, "base64"));
    const L = info.pieceLength, bad = new Set(d.unreadable), wrong = new Set(d.wrong);
    const storage = {{
      async get(offset, length) {{
        await new Promise((r) => setImmediate(r));
        const i = Math.floor(offset / L);
        if (bad.has(i) || offset + length > payload.length) return null;
        const b = payload.slice(offset, offset + length);
        if (!wrong.has(i)) return b;
        const longer = new Uint8Array(length + 1);
        longer.set(b);
        return longer;
      }},
    }};
    const per = [];
    for (const n of [1, 3]) {{
      await m.releaseContexts();
      Deno.fakeReset();
      const bf = await m.verifyStream(info, storage, {{ devices: Array(n).fill(0), chunk: d.chunk }});
      let bits = "";
      for (let i = 0; i < pieces.length; i++) bits += (bf[i >> 3] >> (7 - (i % 8))) & 1;
      per.push(bits);
    }}
    res.push(per);
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    got = json.loads(out)
    for seed, g, w in zip(SEEDS, got, want):
        assert g == [w, w], (seed, g, w)


def test_verify_pieces_host_logic_on_cpu(tmp_path):
    """verifyPieces' host side (batches of storage.get, the availability bits, the staged ranges, shard
    concatenation) on CPU against the JS model of the library for the 48 seeded fuzz layouts on 1 and 3
    shards, with batches of 3 pieces, unreadable pieces and reads one byte too long (unreadable, never
    shifting a later piece): the bits equal hashlib over Storage.get's bytes."""
    from tests.test_gpu_fuzz import SEEDS, _draw
    from torrent_amd.piece import piece_length
    import random as _random
    mod = erased_module(tmp_path)
    spec, want = [], []
    for seed in SEEDS:
        info, payload = _draw(seed)[:2]
        P, L, total = info.n_pieces, info.piece_length, info.length
        rng = _random.Random(seed + 7)
        unreadable = sorted(rng.sample(range(P), min(2, P)))
        wrong = sorted(rng.sample(range(P), 1))
        spec.append({"info": _info_json(L, total, info.pieces_raw), "payload": _b64(payload[:total]),
                     "unreadable": unreadable, "wrong": wrong})
        bits = ""
        for i in range(P):
            n = piece_length(i, info)
            d = info.pieces_raw[20 * i:20 * i + 20]
            ok = (i not in unreadable and i not in wrong and i * L + n <= total and len(d) == 20 and
                  hashlib.sha1(payload[i * L:i * L + n]).digest() == d)
            bits += "1" if ok else "0"
        want.append(bits)
    (tmp_path / "spec.json").write_text(json.dumps(spec))
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const fs = require("fs");
import("{mod}").then(async (m) => {{
  const spec = JSON.parse(fs.readFileSync("{tmp_path}/spec.json", "utf8"));
  const res = [];
  for (const d of spec) {{
    const raw = Buffer.from(d.info.pieces, "base64");
    const pieces = [];
    for (let i = 0; i < raw.length; i += 20) pieces.push(new Uint8Array(raw.subarray(i, Math.min(raw.length, i + 20))));
    const info = {{ pieceLength: d.info.pieceLength, length: d.info.length, pieces, name: "t", private: 0 }};
    const payload = new Uint8Array(Buffer.from(d.payload, "base64"));
    const L = info.pieceLength, bad = new Set(d.unreadable), wrong = new Set(d.wrong);
    const storage = {{
      async get(offset, length) {{
        await new Promise((r) => setImmediate(r));
        const i = Math.floor(offset / L);
        if (bad.has(i) || offset + length > payload.length) return null;
        const b = payload.slice(offset, offset + length);
        if (!wrong.has(i)) return b;
        const longer = new Uint8Array(length + 1);
        longer.set(b);
        longer[length] = 0x5a;
        return longer;
      }},
    }};
    const per = [];
    for (const n of [1, 3]) {{
      await m.releaseContexts();
      Deno.fakeReset();
      const bf = await m.verifyPieces(info, storage, {{ devices: Array(n).fill(0), batchBytes: 3 * L }});
      let bits = "";
      for (let i = 0; i < pieces.length; i++) bits += (bf[i >> 3] >> (7 - (i % 8))) & 1;
      per.push(bits);
    }}
    res.push(per);
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    got = json.loads(out)
    for seed, g, w in zip(SEEDS, got, want):
        assert g == [w, w], (seed, g, w)


def test_reads_in_flight_are_bounded_and_resends_during_a_stage_are_ignored(tmp_path):
    """verifyPieces with its default 256 MiB batch over 600 pieces of 16 KiB, and verifyStream over the same
    torrent, keep at most 32 storage.get calls pending (each fsStorage.get is a Deno.open: a whole batch at once
    would hit EMFILE, and fsStorage.get turns that into null, a valid piece reported 0), and still return every
    piece's bit.  PieceVerifier: a re-sent block of a piece that arrives while the piece's completing stage is
    still pending (nonblocking tv_stage) neither writes into the bytes being copied nor queues the piece twice.
    CPU, against the JS model of the library (tests/ts_harness/fake_deno.js)."""
    mod = erased_module(tmp_path)
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const crypto = require("crypto");
import("{mod}").then(async (m) => {{
  const L = 16384, P = 600, total = L * (P - 1) + 77;
  const payload = crypto.randomBytes(total);
  const pieces = [];
  for (let i = 0; i < P; i++) pieces.push(crypto.createHash("sha1").update(payload.slice(i * L, (i + 1) * L)).digest());
  const info = {{ pieceLength: L, length: total, pieces, name: "t", private: 0 }};
  let inFlight = 0, maxInFlight = 0, calls = 0;
  const storage = {{
    async get(offset, length) {{
      inFlight++; calls++;
      maxInFlight = Math.max(maxInFlight, inFlight);
      await new Promise((r) => setTimeout(r, 1));
      inFlight--;
      return offset + length > payload.length ? null : payload.slice(offset, offset + length);
    }},
  }};
  const ones = (bf) => Array.from({{ length: P }}, (_, i) => (bf[i >> 3] >> (7 - (i % 8))) & 1).join("");
  const res = {{}};
  Deno.fakeReset();
  res.pieces = {{ bits: ones(await m.verifyPieces(info, storage)), max: maxInFlight, calls }};
  maxInFlight = 0; calls = 0;
  await m.releaseContexts();
  Deno.fakeReset();
  res.stream = {{ bits: ones(await m.verifyStream(info, storage, {{ chunk: 4096 }})), max: maxInFlight, calls }};
  // PieceVerifier: the completing block of piece 5 and a corrupted re-send of its first block, concurrently
  const L2 = 32768, info2 = {{ pieceLength: L2, length: 8 * L2, name: "t2", private: 0, pieces: [] }};
  for (let i = 0; i < 8; i++) info2.pieces.push(crypto.createHash("sha1").update(payload.slice(i * L2, (i + 1) * L2)).digest());
  const pv = new m.PieceVerifier(info2, {{ flushPieces: null, flushAgeMs: null }});
  await pv.onBlock(5, 0, payload.slice(5 * L2, 5 * L2 + 16384));
  const done = pv.onBlock(5, 16384, payload.slice(5 * L2 + 16384, 6 * L2));
  const resend = pv.onBlock(5, 0, Buffer.alloc(16384));
  res.verifier = {{ done: await done, resend: await resend, flush: await pv.flush() }};
  await pv.close();
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    assert res["pieces"]["bits"] == "1" * 600 and res["pieces"]["calls"] == 600
    assert 1 < res["pieces"]["max"] <= 32, res["pieces"]
    assert res["stream"]["bits"] == "1" * 600
    assert 1 < res["stream"]["max"] <= 32, res["stream"]
    assert res["verifier"] == {"done": True, "resend": False, "flush": [[5, True]]}


def test_hash_pieces_shards_like_the_python_host(tmp_path):
    """hashPieces shards the pieces over opts.devices as verifyPieces does (and torrent_amd.hash_pieces): each
    shard stages only its own bytes and its digests land at 20 * first -- on 1, 2 and 3 shards, with a short
    last piece and shard boundaries inside the payload, the `pieces` string equals hashlib's.  CPU, against
    the JS model of the library."""
    mod = erased_module(tmp_path)
    L, P = 4096, 37
    payload = random.Random(11).randbytes(L * (P - 1) + 1234)
    want = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    (tmp_path / "payload.bin").write_bytes(payload)
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const fs = require("fs");
import("{mod}").then(async (m) => {{
  const payload = new Uint8Array(fs.readFileSync("{tmp_path}/payload.bin"));
  const res = {{}};
  for (const n of [1, 2, 3]) {{
    await m.releaseContexts();
    Deno.fakeReset();
    res[n] = Buffer.from(await m.hashPieces(payload, {L}, {{ devices: Array(n).fill(0) }})).toString("hex");
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    assert res == {"1": want.hex(), "2": want.hex(), "3": want.hex()}


def test_piece_verifier_slots_shard_and_flush_ordering_on_cpu(tmp_path):
    """PieceVerifier on CPU against the JS model of the library:
    * slot pool: slots = 3 with the caller flushing holds at most 3 staged pieces, forces a flush when a 4th
      completes, and delivers every result once;
    * shard: a verifier over pieces [8, 16) takes only their blocks (a block of piece 3 throws) and lays out
      that shard;
    * flush() called while an automatic (timer) flush is still in its tv_verify_list (a slow call) returns that
      flush's results too (they used to stay behind for a later flush), and poll() hands out what
      automatic flushes returned."""
    mod = erased_module(tmp_path)
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const crypto = require("crypto");
const sleep = (ms) => new Promise((r) => setTimeout(r, ms));
import("{mod}").then(async (m) => {{
  const L = 32768, P = 20, total = L * P;
  const payload = crypto.randomBytes(total);
  const pieces = [];
  for (let i = 0; i < P; i++) pieces.push(crypto.createHash("sha1").update(payload.slice(i * L, (i + 1) * L)).digest());
  const info = {{ pieceLength: L, length: total, pieces, name: "t", private: 0 }};
  const blocksOf = (i) => [0, 16384].map((o) => [i, o, payload.slice(i * L + o, i * L + o + 16384)]);
  const res = {{}};
  {{
    const got = [];
    const pv = new m.PieceVerifier(info, {{ flushPieces: null, flushAgeMs: null, slots: 3, onVerified: (i, ok) => got.push([i, ok]) }});
    for (let i = 0; i < 10; i++) for (const [x, o, b] of blocksOf(i)) await pv.onBlock(x, o, b);
    const fin = await pv.flush();
    const c = [...Deno.fakeContexts.values()].pop();
    res.slots = {{ forced: pv.forcedFlushes, slots: pv.slots, max: c.maxStaged, opt: c.options[17], all: [...got, ...fin] }};
    await pv.close();
  }}
  {{
    const pv = new m.PieceVerifier(info, {{ shard: [8, 8], flushPieces: 2, flushAgeMs: null }});
    const c = [...Deno.fakeContexts.values()].pop();
    let threw = false;
    try {{ await pv.onBlock(3, 0, payload.slice(3 * L, 3 * L + 16384)); }} catch (e) {{ threw = true; }}
    for (let i = 8; i < 12; i++) for (const [x, o, b] of blocksOf(i)) await pv.onBlock(x, o, b);
    const polled = await pv.poll();
    res.shard = {{ threw, first: c.first, count: c.count, polled, fin: await pv.flush(), slots: pv.slots }};
    let bad = false;
    try {{ new m.PieceVerifier(info, {{ shard: [4, 8] }}); }} catch (e) {{ bad = true; }}
    res.shard.badShardThrows = bad;
    await pv.close();
  }}
  {{
    Deno.fakeDelayMs = 20;
    const pv = new m.PieceVerifier(info, {{ flushPieces: null, flushAgeMs: 1 }});
    for (const [x, o, b] of blocksOf(0)) await pv.onBlock(x, o, b);   // staged by ~20 ms; timer 1 ms later
    await sleep(8);                                                    // the timer's flush is in tv_verify_list
    const fin = await pv.flush();
    res.order = {{ fin, autoFlushes: pv.autoFlushes }};
    Deno.fakeDelayMs = 0;
    await pv.close();
  }}
  {{
    // close() while the age timer's flush is inside its (slow) tv_verify_list: the context is destroyed only after
    // it returns, its results still reach onVerified, and the verifier refuses further use
    Deno.fakeDelayMs = 20;
    const got = [];
    const pv = new m.PieceVerifier(info, {{ flushPieces: null, flushAgeMs: 1, onVerified: (i, ok) => got.push([i, ok]) }});
    for (const [x, o, b] of blocksOf(1)) await pv.onBlock(x, o, b);
    await sleep(8);
    await pv.close();
    let threw = false;
    try {{ await pv.onBlock(2, 0, payload.slice(2 * L, 2 * L + 16384)); }} catch (e) {{ threw = /closed/.test(String(e)); }}
    Deno.fakeDelayMs = 0;
    res.close = {{ got, violations: Deno.fakeViolations.slice(), threw }};
  }}
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    assert res["slots"]["forced"] == 3 and res["slots"]["max"] == 3 and res["slots"]["slots"] == 3
    assert res["slots"]["opt"] == 3
    assert res["slots"]["all"] == [[i, True] for i in range(10)]
    assert res["shard"]["threw"] and res["shard"]["first"] == 8 and res["shard"]["count"] == 8
    assert res["shard"]["polled"] == [[8, True], [9, True], [10, True], [11, True]] and res["shard"]["fin"] == []
    assert res["shard"]["slots"] == 2 and res["shard"]["badShardThrows"]
    assert res["close"] == {"got": [[1, True]], "violations": [], "threw": True}
    assert res["order"] == {"fin": [[0, True]], "autoFlushes": 1}


def test_binding_stays_within_its_minimum_deno(tmp_path):
    """ts/verify.ts states its minimum Deno (1.31: pointer objects, UnsafePointer.create / value; nonblocking
    symbols): its code uses no Deno member outside that version's FFI surface (tests/ts_harness/deno_api.js), its
    whole symbol table passes the harness's 1.31 check (both shims apply it at dlopen), and a table using a newer
    FFI feature -- a struct type (1.35), an `optional` symbol (1.36), a "bool" result -- is rejected."""
    import re
    src = open(os.path.join(ROOT, "ts", "verify.ts")).read()
    assert "Deno 1.31" in src.split("\nimport ")[0]                              # the header states it
    assert "1.31" in open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    code = "\n".join(line.split("//")[0] for line in code.splitlines())         # (no // inside strings here)
    used = set(re.findall(r"Deno\.([A-Za-z]+(?:\.[A-Za-z]+)?)", code))
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const api = require("./deno_api.js");
const res = {{ surface: api.SURFACE, min: api.MIN_VERSION, rejected: [] }};
const probes = {{
  struct: {{ f: {{ parameters: [{{ struct: ["u8", "u32"] }}], result: "void" }} }},
  optional: {{ f: {{ parameters: [], result: "i32", optional: true }} }},
  bool: {{ f: {{ parameters: [], result: "bool" }} }},
}};
for (const [k, table] of Object.entries(probes)) {{
  try {{ Deno.dlopen("x", table); }} catch (e) {{ res.rejected.push(k); }}
}}
import("{erased_module(tmp_path)}").then(async (m) => {{
  // the binding's own table binds through the checked dlopen (a zero-piece call loads it)
  const info = {{ pieceLength: 16384, length: 0, pieces: [], name: "t", private: 0 }};
  res.bound = (await m.verifyPieces(info, {{ async get() {{ return null; }} }})).length === 0;
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    assert res["min"] == "1.31" and res["bound"]
    assert sorted(res["rejected"]) == ["bool", "optional", "struct"]
    assert used <= set(res["surface"]), used - set(res["surface"])


def test_opt_in_cpu_path_on_cpu(tmp_path):
    """The opt-in CPU path runs the reference's own crypto.subtle.digest("SHA-1", ...)
    (tools/make_torrent.ts:28-31; here Node's SHA-1 stands in for WebCrypto, which Node 12 lacks): verifyPiece
    with cpuFallback never loads the library (a missing libPath still answers) and gives hashlib's answer;
    PieceVerifier with cpuFallbackMaxPieces = 3 hashes a flush of <= 3 pieces on the CPU (no list launch, nothing
    staged) and sends a longer one to the library (staged at the flush, one tv_verify_list), with identical bits
    either way, a corrupted piece included.  Off by default."""
    mod = erased_module(tmp_path)
    out = run_node(tmp_path, f"""
import {{ createRequire }} from "module";
const require = createRequire("{HARNESS}/");
const Deno = require("./fake_deno.js");
const nodeCrypto = require("crypto");
globalThis.crypto = {{ subtle: {{ async digest(alg, data) {{
  if (alg !== "SHA-1") throw new Error(alg);
  const b = nodeCrypto.createHash("sha1").update(Buffer.from(data)).digest();
  return b.buffer.slice(b.byteOffset, b.byteOffset + 20);
}} }} }};
import("{mod}").then(async (m) => {{
  const L = 32768, P = 12, total = L * P;
  const payload = nodeCrypto.randomBytes(total);
  const pieces = [];
  for (let i = 0; i < P; i++) pieces.push(nodeCrypto.createHash("sha1").update(payload.slice(i * L, (i + 1) * L)).digest());
  const info = {{ pieceLength: L, length: total, pieces, name: "t", private: 0 }};
  const res = {{}};
  res.piece = [await m.verifyPiece(info, 3, payload.slice(3 * L, 4 * L), {{ cpuFallback: true, libPath: "/nonexistent.so" }}),
               await m.verifyPiece(info, 3, Buffer.alloc(L), {{ cpuFallback: true, libPath: "/nonexistent.so" }})];
  const pv = new m.PieceVerifier(info, {{ flushPieces: null, flushAgeMs: null, cpuFallbackMaxPieces: 3 }});
  const c = [...Deno.fakeContexts.values()].pop();
  const feed = async (i, bad) => {{
    for (const o of [0, 16384]) {{
      const b = Buffer.from(payload.slice(i * L + o, i * L + o + 16384));
      if (bad && o === 0) b[7] ^= 1;
      await pv.onBlock(i, o, b);
    }}
  }};
  await feed(0); await feed(1, true);
  res.short = {{ out: await pv.flush(), lists: c.lists || 0, staged: c.staged.size }};
  for (let i = 2; i < 7; i++) await feed(i, i === 5);
  res.long = {{ out: await pv.flush(), lists: c.lists || 0 }};
  res.bits = Array.from({{ length: P }}, (_, i) => (pv.bitfield[i >> 3] >> (7 - (i % 8))) & 1).join("");
  await pv.close();
  console.log(JSON.stringify(res));
}}).catch((e) => {{ console.error(e); process.exit(1); }});
""")
    res = json.loads(out)
    assert res["piece"] == [True, False]
    assert res["short"] == {"out": [[0, True], [1, False]], "lists": 0, "staged": 0}
    assert res["long"] == {"out": [[2, True], [3, True], [4, True], [5, False], [6, True]], "lists": 1}
    assert res["bits"] == "101110100000"
