"""Where ts/verify.ts verifyFiles spends its time on a layout (type-erased, under Node 12 with the Deno FFI shim of
tests/ts_harness, on the GPU): Deno.dlopen is wrapped so every library call made during the call is timed (the
nonblocking ones from the call to the settled promise), and the rest of the wall time is the host's own JavaScript.
Runs verifyFiles `reps` times after one warm-up call and prints one JSON line per call.

    python tools/ts_files_phases.py DIR [cfg3|single16|files64] [reps]
"""
import json
import os
import shutil
import subprocess
import sys

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
const times = {};
const add = (k, ns) => { times[k] = (times[k] || 0) + ns; };
const realOpen = Deno.dlopen;
Deno.dlopen = (p, syms) => {
  const lib = realOpen(p, syms);
  const out = {};
  for (const [name, fn] of Object.entries(lib.symbols)) {
    out[name] = (...a) => {
      const t0 = process.hrtime.bigint();
      const r = fn(...a);
      if (r && typeof r.then === "function") {
        return r.then((v) => { add(name, Number(process.hrtime.bigint() - t0)); return v; });
      }
      add(name, Number(process.hrtime.bigint() - t0));
      return r;
    };
  }
  return { symbols: out, close: () => lib.close() };
};
import(pathToFileURL("MODULE").href).then(async (v) => {
  const spec = JSON.parse(fs.readFileSync("SPEC", "utf8"));
  const raw = Buffer.from(spec.pieces, "base64");
  const pieces = [];
  for (let i = 0; i < raw.length; i += 20) pieces.push(new Uint8Array(raw.subarray(i, i + 20)));
  const info = { pieceLength: spec.pieceLength, length: spec.length, pieces, name: spec.name, private: 0 };
  if (spec.files) info.files = spec.files;
  const opts = { libPath: spec.lib };
  const hex = (u8) => Buffer.from(u8).toString("hex");
  for (let r = 0; r <= REPS; r++) {
    for (const k of Object.keys(times)) delete times[k];
    const t0 = process.hrtime.bigint();
    const bf = await v.verifyFiles(info, spec.dir, opts);
    const wall = Number(process.hrtime.bigint() - t0);
    let lib = 0;
    const calls = {};
    for (const [k, ns] of Object.entries(times)) { lib += ns; calls[k] = +(ns / 1e6).toFixed(3); }
    console.log(JSON.stringify({ layout: spec.layout, rep: r, warmup: r === 0, wall_ms: +(wall / 1e6).toFixed(2),
                                 gbps: +(spec.length / wall).toFixed(2), exact: hex(bf) === spec.expect,
                                 library_calls_ms: calls, host_js_ms: +((wall - lib) / 1e6).toFixed(2) }));
  }
  await v.releaseContexts();
}).catch((e) => { console.error(e); process.exit(1); });
"""


def main():
    d = sys.argv[1]
    layout = sys.argv[2] if len(sys.argv) > 2 else "cfg3"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    node = shutil.which("node")
    mod = os.path.join(d, "verify.mjs")
    os.makedirs(d, exist_ok=True)
    with open(mod, "w") as f:
        f.write(erase(open(os.path.join(ROOT, "ts", "verify.ts")).read()))
    root = os.path.join(d, layout)
    info, expect, _ = write_layout(layout, root)
    spec = {"layout": layout, "pieceLength": info.piece_length, "length": info.length, "name": info.name,
            "pieces": __import__("base64").b64encode(info.pieces_raw).decode(), "dir": root,
            "expect": bytes(expect).hex(), "lib": os.path.join(ROOT, "torrent_amd", "libtorrent_verify.so")}
    if info.files is not None:
        spec["files"] = [{"length": f.length, "path": list(f.path)} for f in info.files]
    sp = os.path.join(d, f"spec_{layout}.json")
    with open(sp, "w") as f:
        json.dump(spec, f)
    script = os.path.join(d, "phases.mjs")
    with open(script, "w") as f:
        f.write(SCRIPT.replace("HARNESS", HARNESS).replace("MODULE", mod).replace("SPEC", sp)
                .replace("REPS", str(reps)))
    r = subprocess.run([node, script], capture_output=True, text=True, cwd=HARNESS, timeout=600)
    sys.stdout.write(r.stdout)
    if r.returncode:
        sys.stderr.write(r.stderr)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
