// fake_deno.js -- a CPU model of the library behind the Deno FFI, for the TS host logic on CPU (test
// infrastructure only; tests/test_ts_binding.py).  Deno.dlopen returns JavaScript implementations of the
// calls PieceVerifier makes (tv_create / tv_set_layout / tv_set_digests / tv_stage / tv_verify_list /
// tv_destroy / tv_last_error / tv_abi_version), with SHA-1 from node's crypto as the checker; every other
// symbol throws if called.  Pointers are the typed arrays themselves.  `nonblocking` symbols resolve on a
// later turn of the event loop, as Deno's do, so the verifier's timer and its block handler interleave.
"use strict";
const crypto = require("crypto");

const contexts = new Map();
let nextHandle = 1n;

function bytesOf(p) {
  return p instanceof Uint8Array ? p : new Uint8Array(p.buffer, p.byteOffset, p.byteLength);
}

const impl = {
  tv_abi_version: () => 1,
  tv_create(out) {
    const h = nextHandle++;
    new BigUint64Array(bytesOf(out).buffer, bytesOf(out).byteOffset, 1)[0] = h;
    contexts.set(h, { staged: new Map() });
    return 0;
  },
  tv_set_layout(ctx, total, L, P, first, count) {
    Object.assign(contexts.get(ctx), { total: Number(total), L: Number(L), P: Number(P), first: Number(first),
                                       count: Number(count), staged: new Map() });
    return 0;
  },
  tv_set_digests(ctx, p, n) {
    contexts.get(ctx).digests = Buffer.from(bytesOf(p).slice(0, Number(n)));
    return 0;
  },
  tv_stage(ctx, off, p, n) {
    const c = contexts.get(ctx);
    const i = Number(off) / c.L;
    c.staged.set(i, Buffer.from(bytesOf(p).slice(0, Number(n))));
    return 0;
  },
  tv_verify_list(ctx, idxp, n, okp) {
    const c = contexts.get(ctx);
    const b = bytesOf(idxp);
    const idx = new BigUint64Array(b.buffer, b.byteOffset, Number(n));
    const ok = bytesOf(okp);
    c.lists = (c.lists || 0) + 1;
    idx.forEach((v, k) => {
      const i = Number(v);
      const data = c.staged.get(i);
      const d = c.digests.slice(20 * i, 20 * i + 20);
      ok[k] = data && d.length === 20 && crypto.createHash("sha1").update(data).digest().equals(d) ? 1 : 0;
    });
    return 0;
  },
  tv_destroy(ctx) {
    contexts.delete(ctx);
  },
  tv_last_error: () => 0,
};

const Deno = {
  dlopen(_path, symbols) {
    const out = {};
    for (const name of Object.keys(symbols)) {
      const f = impl[name] || (() => {
        throw new Error(`fake_deno: ${name} is not modelled`);
      });
      out[name] = symbols[name].nonblocking
        ? (...a) => new Promise((res, rej) => setImmediate(() => {
          try {
            res(f(...a));
          } catch (e) {
            rej(e);
          }
        }))
        : f;
    }
    return { symbols: out, close() {} };
  },
  UnsafePointer: { of: (ta) => ta, create: (v) => (v === 0n ? null : v), value: (p) => p },
  UnsafePointerView: {},
  fakeContexts: contexts,
};

globalThis.Deno = Deno;
if (typeof globalThis.performance === "undefined") globalThis.performance = require("perf_hooks").performance;
module.exports = Deno;
