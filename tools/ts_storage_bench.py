"""The TypeScript host's Storage paths, measured: ts/verify.ts (type-erased, under Node 12 with the Deno FFI shim of
tests/ts_harness, on the GPU) runs verifyPieces / verifyStream over a JS restatement of the reference's `Storage` +
`fsStorage` (storage.ts:50-65,89-137,149-172: every get opens the file read + write, reads, closes -- here through
Node's fs, whose work runs on libuv's thread pool as Deno's ops run on its blocking pool) and verifyFiles over the
same directory.  Every bitfield is compared with hashlib's / the committed bits.

    python tools/ts_storage_bench.py DIR [single16|files64|cfg3 ...]      (env UV_THREADPOOL_SIZE: libuv's pool;
                                                                           TS_SRC: another verify.ts, for A/Bs)

One JSON line per (layout, path): best wall seconds of 2 runs, GB/s, exact."""
import base64
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
HARNESS = os.path.join(ROOT, "tests", "ts_harness")
sys.path.insert(0, HARNESS)
from erase_ts import erase  # noqa: E402
from storage_paths_bench import write_layout  # noqa: E402

SCRIPT = r"""
import { createRequire } from "module";
import { pathToFileURL } from "url";
const require = createRequire("HARNESS/");
require("./deno_shim.js");
const fs = require("fs");
const path = require("path");

// fsStorage (storage.ts:149-172): open read + write + create, seek, read exactly `length`, close; null on failure
const fsStorage = {
  async get(p, offset, length) {
    let fh = null;
    try {
      fh = await fs.promises.open(path.join(...p), fs.constants.O_RDWR | fs.constants.O_CREAT);
      const buf = new Uint8Array(length);
      let got = 0;
      while (got < length) {
        const { bytesRead } = await fh.read(buf, got, length - got, offset + got);
        if (bytesRead === 0) break;
        got += bytesRead;
      }
      await fh.close();
      return got === length ? buf : null;
    } catch (e) {
      if (fh) try { await fh.close(); } catch (e2) { /* nothing */ }
      return null;
    }
  },
};

// Storage.get (storage.ts:50-65 over findAndDo, :89-137): the file segments of [offset, offset + length) in order
function makeStorage(info, dir) {
  const files = info.files ? info.files.map((f) => ({ length: f.length, path: [dir, ...f.path] }))
                           : [{ length: info.length, path: [dir, info.name] }];
  const starts = [];
  let acc = 0;
  for (const f of files) { starts.push(acc); acc += f.length; }
  return {
    async get(offset, length) {
      const out = new Uint8Array(length);
      let k = 0;
      while (k < files.length && starts[k] + files[k].length <= offset && !(files[k].length === 0 && starts[k] === offset)) k++;
      let pos = offset;
      const end = offset + length;
      for (; k < files.length && pos < end; k++) {
        const f = files[k];
        const foff = pos - starts[k];
        const n = Math.min(f.length - foff, end - pos);
        if (n < 0) continue;
        const got = await fsStorage.get(f.path, foff, n);
        if (got === null) return null;
        out.set(got, pos - offset);
        pos += n;
      }
      return pos === end ? out : null;
    },
  };
}

const hex = (u8) => Buffer.from(u8).toString("hex");
import(pathToFileURL("MODULE").href).then(async (v) => {
  const spec = JSON.parse(fs.readFileSync("SPEC", "utf8"));
  const raw = Buffer.from(spec.pieces, "base64");
  const pieces = [];
  for (let i = 0; i < raw.length; i += 20) pieces.push(new Uint8Array(raw.subarray(i, i + 20)));
  const info = { pieceLength: spec.pieceLength, length: spec.length, pieces, name: spec.name, private: 0 };
  if (spec.files) info.files = spec.files;
  const st = makeStorage(info, spec.dir);
  const opts = { libPath: spec.lib };
  // the reads alone, as the binding issues them (32 in flight, bytes dropped): the Storage restatement, and for a
  // single-file torrent fsStorage.get itself (no Storage copy)
  const P = pieces.length, L = info.pieceLength;
  const plen = (i) => (i === P - 1 && info.length % L ? info.length % L : L);
  const readAll = async (get) => {
    let next = 0;
    const worker = async () => { while (next < P) { const i = next++; await get(i); } };
    await Promise.all(Array.from({ length: 32 }, worker));
    return new Uint8Array(0);
  };
  const readLegs = [["Storage.get only (32 in flight)", () => readAll((i) => st.get(i * L, plen(i)))]];
  if (!info.files) {
    readLegs.push(["fsStorage.get only (32 in flight)", () => readAll((i) => fsStorage.get([spec.dir, info.name], i * L, plen(i)))]);
  }
  for (const [name, fn] of readLegs) {
    let best = Infinity;
    for (let r = 0; r < 2; r++) {
      const t0 = process.hrtime.bigint();
      await fn();
      best = Math.min(best, Number(process.hrtime.bigint() - t0) / 1e9);
    }
    console.log(JSON.stringify({ layout: spec.layout, path: name, best_s: +best.toFixed(4),
                                 gbps: +(spec.length / best / 1e9).toFixed(2),
                                 uv_threadpool: process.env.UV_THREADPOOL_SIZE || "4 (default)" }));
  }
  const legs = [["verifyPieces", () => v.verifyPieces(info, st, opts)],
                ["verifyStream rows", () => v.verifyStream(info, st, opts)],
                ["verifyFiles", () => v.verifyFiles(info, spec.dir, opts)]];
  for (const [name, fn] of legs) {
    let best = Infinity, exact = true;
    for (let r = 0; r < 2; r++) {
      const t0 = process.hrtime.bigint();
      const bf = await fn();
      const el = Number(process.hrtime.bigint() - t0) / 1e9;
      exact = exact && hex(bf) === spec.expect;
      best = Math.min(best, el);
    }
    console.log(JSON.stringify({ layout: spec.layout, path: name, best_s: +best.toFixed(4),
                                 gbps: +(spec.length / best / 1e9).toFixed(2), exact,
                                 uv_threadpool: process.env.UV_THREADPOOL_SIZE || "4 (default)" }));
  }
  await v.releaseContexts();
}).catch((e) => { console.error(e); process.exit(1); });
"""


def main():
    d = sys.argv[1]
    node = shutil.which("node")
    mod = os.path.join(d, "verify.mjs")
    os.makedirs(d, exist_ok=True)
    with open(mod, "w") as f:
        f.write(erase(open(os.environ.get("TS_SRC") or os.path.join(ROOT, "ts", "verify.ts")).read()))
    for layout in sys.argv[2:] or ["single16"]:
        root = os.path.join(d, layout)
        info, expect, _ = write_layout(layout, root)
        spec = {"layout": layout, "pieceLength": info.piece_length, "length": info.length, "name": info.name,
                "pieces": base64.b64encode(info.pieces_raw).decode(), "dir": root, "expect": bytes(expect).hex(),
                "lib": os.path.join(ROOT, "torrent_amd", "libtorrent_verify.so")}
        if info.files is not None:
            spec["files"] = [{"length": f.length, "path": list(f.path)} for f in info.files]
        sp = os.path.join(d, f"spec_{layout}.json")
        with open(sp, "w") as f:
            json.dump(spec, f)
        script = os.path.join(d, "bench.mjs")
        with open(script, "w") as f:
            f.write(SCRIPT.replace("HARNESS", HARNESS).replace("MODULE", mod).replace("SPEC", sp))
        t0 = time.perf_counter()
        r = subprocess.run([node, script], capture_output=True, text=True, cwd=HARNESS, timeout=900)
        sys.stdout.write(r.stdout)
        if r.returncode:
            sys.stderr.write(r.stderr)
            return r.returncode
        print(json.dumps({"layout": layout, "node_wall_s": round(time.perf_counter() - t0, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
