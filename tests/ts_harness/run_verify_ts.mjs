// run_verify_ts.mjs -- run ts/verify.ts (type-erased by erase_ts.py) under Node 12 with the Deno FFI shim,
// against the real libtorrent_verify.so.  Test infrastructure only (tests/test_ts_binding.py).
//
//   node run_verify_ts.mjs <verify.mjs> <spec.json> <out.json>
//
// spec.cases[k].kind:
//   "pieces"   verifyPieces(info, storage)       storage = the linear payload, minus unreadable pieces
//   "stream"   verifyStream(info, storage)       (rows of `wrongLength` pieces come back one byte long)
//   "files"    verifyFiles(info, dir) (stream / budget: the streamed-columns form under a device budget)
//   "piece"    verifyPiece(info, index, bytes)
//   "hash"     hashPieces(payload, pieceLength)
//   "verifier" PieceVerifier: onBlock per block, automatic flushes (onVerified), optionally `settleMs` of
//              idle time for the age timer, then flush()
// Bytes travel as base64.  Every result goes to out.json; the Python side compares.
import { createRequire } from "module";
import { pathToFileURL } from "url";
import fs from "fs";

const require = createRequire(import.meta.url);
require("./deno_shim.js");

const b64 = (s) => new Uint8Array(Buffer.from(s, "base64"));
const hex = (u8) => Buffer.from(u8).toString("hex");

function makeInfo(d) {
  const raw = b64(d.pieces);
  const pieces = [];
  for (let i = 0; i < raw.length; i += 20) pieces.push(raw.subarray(i, Math.min(raw.length, i + 20)));
  const info = { pieceLength: d.pieceLength, length: d.length, pieces, name: d.name, private: 0 };
  if (d.files) info.files = d.files;
  return info;
}

function memStorage(payload, L, unreadable, wrongLength) {
  const bad = new Set(unreadable || []);
  const wrong = new Set(wrongLength || []);
  return {
    async get(offset, length) {
      const piece = Math.floor(offset / L);
      if (bad.has(piece) || offset + length > payload.length) return null;
      if (wrong.has(piece)) return payload.slice(offset, offset + Math.max(1, length - 1));
      return payload.slice(offset, offset + length);
    },
  };
}

async function main() {
  const [modPath, specPath, outPath] = process.argv.slice(2);
  const v = await import(pathToFileURL(modPath).href);
  const spec = JSON.parse(fs.readFileSync(specPath, "utf8"));
  const opts = { libPath: spec.lib };
  const out = [];
  for (const c of spec.cases) {
    const r = { name: c.name, kind: c.kind };
    try {
      if (c.kind === "pieces" || c.kind === "stream") {
        const info = makeInfo(c.info);
        const st = memStorage(b64(c.payload), c.info.pieceLength, c.unreadable, c.wrongLength);
        const o = { ...opts, devices: c.devices };
        r.bitfield = hex(c.kind === "pieces" ? await v.verifyPieces(info, st, o) : await v.verifyStream(info, st, { ...o, chunk: c.chunk || 0 }));
      } else if (c.kind === "files") {
        r.bitfield = hex(await v.verifyFiles(makeInfo(c.info), c.dir,
                                             { ...opts, devices: c.devices, stream: c.stream, budget: c.budget }));
      } else if (c.kind === "piece") {
        r.ok = await v.verifyPiece(makeInfo(c.info), c.index, b64(c.bytes), opts);
      } else if (c.kind === "hash") {
        r.pieces = hex(await v.hashPieces(b64(c.payload), c.pieceLength, { ...opts, devices: c.devices }));
      } else if (c.kind === "verifier") {
        const got = [];
        const pv = new v.PieceVerifier(makeInfo(c.info), {
          ...opts, flushPieces: c.flushPieces, flushAgeMs: c.flushAgeMs, onVerified: (i, ok) => got.push([i, ok]),
        });
        let completed = 0;
        for (const [index, offset, data] of c.blocks) if (await pv.onBlock(index, offset, b64(data))) completed++;
        // the age bound also fires without further blocks (its timer): let it
        if (c.settleMs) await new Promise((res) => setTimeout(res, c.settleMs));
        r.auto = got.slice();
        r.autoFlushes = pv.autoFlushes;
        r.final = await pv.flush();
        r.completed = completed;
        r.bitfield = hex(pv.bitfield);
        await pv.close();
      } else {
        throw new Error("unknown case kind " + c.kind);
      }
    } catch (e) {
      r.error = String(e && e.stack ? e.stack : e);
    }
    out.push(r);
  }
  await v.releaseContexts();
  fs.writeFileSync(outPath, JSON.stringify(out));
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});
