// fake_deno.js -- a CPU model of the library behind the Deno FFI, for the TS host logic on CPU (test
// infrastructure only; tests/test_ts_binding.py).  Deno.dlopen returns JavaScript implementations of the
// calls PieceVerifier makes (tv_create / tv_set_layout / tv_set_digests / tv_stage(_many) / tv_verify_list /
// tv_destroy / tv_last_error / tv_abi_version) and hashPieces makes (tv_hash), with SHA-1 from node's crypto as the checker, and the
// calls verifyFiles makes (tv_set_option, tv_stage_file_table recording the segment plan the library's own walk makes of
// the host's file table, tv_cpu_share, tv_verify
// returning the host's availability bits) and verifyStream makes (the tv_stream_* protocol, modelled with
// several requests per column); every other symbol throws if called.  Pointers are BigInt
// addresses of registered typed arrays.  `nonblocking` symbols resolve on a
// later turn of the event loop, as Deno's do, so the verifier's timer and its block handler interleave
// (Deno.fakeDelayMs > 0: that many milliseconds later, a slow call).  The slot pool (TV_OPT_LIST_SLOTS) is
// modelled: a staged piece holds a slot until tv_verify_list lists it; staging a new piece with every slot
// taken returns TV_ERR_STATE (-3), as the library does.
"use strict";
const crypto = require("crypto");
const api = require("./deno_api.js");   // the FFI surface of the binding's minimum Deno (1.31)

const contexts = new Map();
let nextHandle = 1n;
// pointers: UnsafePointer.of registers a typed array under a BigInt address, as the real one returns one
const memory = new Map();
let nextAddress = 0x1000n;

function bytesOf(p) {
  let ta = typeof p === "bigint" ? memory.get(p) : p;
  let off = 0;
  if (!ta && typeof p === "bigint") {   // an interior pointer: a registered array's address + an offset into it
    for (const [a, t] of memory) {
      if (p > a && p < a + BigInt(t.byteLength)) {
        ta = t;
        off = Number(p - a);
        break;
      }
    }
  }
  if (!ta) throw new Error("fake_deno: unknown pointer " + p);
  const b = ta instanceof Uint8Array ? ta : new Uint8Array(ta.buffer, ta.byteOffset, ta.byteLength);
  return off ? b.subarray(off) : b;
}

function u64s(p, n) {
  const b = bytesOf(p);
  return new BigUint64Array(b.buffer.slice(b.byteOffset, b.byteOffset + 8 * n));
}

function cString(p) {
  const b = bytesOf(p);
  const end = b.indexOf(0);
  return Buffer.from(b.subarray(0, end < 0 ? b.length : end)).toString("utf8");
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
  // tv_stage: linear bytes [off, off + n) into the staged pieces (a piece's buffer is its pieceLength)
  tv_stage(ctx, off, p, n) {
    const c = contexts.get(ctx);
    const src = bytesOf(p);
    const slots = (c.options && c.options[17]) || 0;
    for (let pos = Number(off), q = 0; q < Number(n);) {
      const i = Math.floor(pos / c.L), within = pos % c.L;
      const plen = i === c.P - 1 && c.total % c.L ? c.total % c.L : c.L;
      if (within >= plen) break;
      const k = Math.min(plen - within, Number(n) - q);
      if (slots && !c.staged.has(i) && c.staged.size >= slots) return -3;
      if (!c.staged.has(i)) c.staged.set(i, Buffer.alloc(plen));
      c.maxStaged = Math.max(c.maxStaged || 0, c.staged.size);
      c.staged.get(i).set(src.subarray(q, q + k), within);
      pos += k;
      q += k;
    }
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
    if ((c.options && c.options[17]) || 0) idx.forEach((v) => c.staged.delete(Number(v)));   // slots freed
    return 0;
  },
  tv_set_option(ctx, key, value) {
    const c = contexts.get(ctx);
    c.options = c.options || {};
    c.options[Number(key)] = Number(value);
    return 0;
  },
  // the stream protocol (tv_stream_*): columns of width C (TV_OPT_STREAM_CHUNK, else the piece length),
  // requests of at most 7 rows so a shard takes several, rows appended per piece and hashed at the end
  tv_stream_begin(ctx, availp) {
    const c = contexts.get(ctx);
    const C = (c.options && c.options[3]) || c.L;
    const reqs = [];
    for (let off = 0; off < c.L; off += C) {
      for (let j = 0; j < c.count; j += 7) reqs.push({ piece: c.first + j, rows: Math.min(7, c.count - j), offset: off, width: C });
    }
    const avail = availp === null ? null : Buffer.from(bytesOf(availp).slice(0, Math.ceil(c.count / 8)));
    c.stream = { reqs, k: 0, data: new Map(), unreadable: new Set(), avail };
    return 0;
  },
  tv_stream_next(ctx, reqp) {
    const c = contexts.get(ctx);
    const st = c.stream;
    const out = new BigUint64Array(bytesOf(reqp).buffer, bytesOf(reqp).byteOffset, 6);
    if (st.k >= st.reqs.length) {
      out.fill(0n);
      return 0;
    }
    const r = st.reqs[st.k];
    const slot = new ArrayBuffer(r.rows * r.width);
    const addr = Deno.UnsafePointer.of(new Uint8Array(slot));
    st.slot = slot;
    out.set([BigInt(r.piece), BigInt(r.rows), BigInt(r.offset), BigInt(r.width), addr, BigInt(st.k)]);
    return 0;
  },
  tv_stream_unreadable(ctx, piece) {
    contexts.get(ctx).stream.unreadable.add(Number(piece));
    return 0;
  },
  tv_stream_commit(ctx) {
    const c = contexts.get(ctx);
    const st = c.stream;
    const r = st.reqs[st.k++];
    const slot = new Uint8Array(st.slot);
    for (let q = 0; q < r.rows; q++) {
      const i = r.piece + q;
      const plen = i === c.P - 1 && c.total % c.L ? c.total % c.L : c.L;
      const n = Math.max(0, Math.min(r.width, plen - r.offset));
      const prev = st.data.get(i) || Buffer.alloc(0);
      st.data.set(i, Buffer.concat([prev, Buffer.from(slot.subarray(q * r.width, q * r.width + n))]));
    }
    return 0;
  },
  tv_stream_end(ctx, outp) {
    const c = contexts.get(ctx);
    const st = c.stream;
    const out = bytesOf(outp);
    out.fill(0, 0, Math.ceil(c.count / 8));
    for (let j = 0; j < c.count; j++) {
      const i = c.first + j;
      const d = c.digests.slice(20 * i, 20 * i + 20);
      const okAvail = !st.avail || (st.avail[j >> 3] >> (7 - (j % 8))) & 1;
      const ok = okAvail && !st.unreadable.has(i) && d.length === 20 &&
        crypto.createHash("sha1").update(st.data.get(i) || Buffer.alloc(0)).digest().equals(d);
      if (ok) out[j >> 3] |= 0x80 >> (j % 8);
    }
    c.stream = null;
    return 0;
  },
  tv_stream_abort(ctx) {
    contexts.get(ctx).stream = null;
    return 0;
  },
  // tv_stage_many: tv_stage of each (offset, buffer address, length) in order
  tv_stage_many(ctx, n, offsp, srcsp, lensp) {
    const view = (p) => {
      const b = bytesOf(p);
      return new BigUint64Array(b.buffer, b.byteOffset, Number(n));
    };
    const offs = view(offsp), srcs = view(srcsp), lens = view(lensp);
    for (let k = 0; k < Number(n); k++) {
      const rc = impl.tv_stage(ctx, offs[k], srcs[k], lens[k]);
      if (rc) return rc;
    }
    return 0;
  },
  // tv_stage_files records the segments it is given (the host's plan) and reports them all readable
  tv_stage_files(ctx, n, pathsp, fop, linp, lenp, statusp) {
    const k = Number(n);
    const paths = u64s(pathsp, k), fo = u64s(fop, k), lin = u64s(linp, k), len = u64s(lenp, k);
    const c = contexts.get(ctx);
    c.segments = c.segments || [];
    for (let q = 0; q < k; q++) c.segments.push([cString(paths[q]), Number(fo[q]), Number(lin[q]), Number(len[q])]);
    new Int32Array(bytesOf(statusp).buffer, bytesOf(statusp).byteOffset, k).fill(0);
    return 0;
  },
  // tv_stage_file_table: the library's own walk of the file table (tv_plan.h walk_file_table, built for the CPU as
  // tests/c/walk_main.cpp; $TV_WALK_EXE) gives the shard's segments, recorded as tv_stage_files records them
  tv_stage_file_table(ctx, n, lensp, pathsp, pathsBytes, statusp) {
    const k = Number(n);
    const c = contexts.get(ctx);
    const lens = u64s(lensp, k);
    const buf = bytesOf(pathsp).subarray(0, Number(pathsBytes));
    const paths = [];
    for (let q = 0, o = 0; q < k; q++) {
      const e = buf.indexOf(0, o);
      if (e < 0) return -2;   // TV_ERR_ARG: fewer than n paths
      paths.push(Buffer.from(buf.subarray(o, e)).toString("utf8"));
      o = e + 1;
    }
    const last = c.first + c.count - 1;
    const plen = last === c.P - 1 && c.total % c.L ? c.total % c.L : c.L;
    const lo = c.first * c.L, hi = Math.min(c.total, last * c.L + plen);
    if (!process.env.TV_WALK_EXE) throw new Error("fake_deno: tv_stage_file_table needs $TV_WALK_EXE");
    const out = require("child_process").execFileSync(process.env.TV_WALK_EXE,
      { input: `${k} ${lo} ${hi} ${c.L}\n${lens.join(" ")}\n` }).toString();
    for (const ln of out.split("\n")) {
      if (!ln || ln.startsWith("reached")) continue;
      const [f, fo, lin, len] = ln.split(" ").map(Number);
      (c.segments = c.segments || []).push([paths[f], fo, lin, len]);
    }
    new Int32Array(bytesOf(statusp).buffer, bytesOf(statusp).byteOffset, k).fill(0);
    return 0;
  },
  tv_cpu_share(outp) {
    new Uint32Array(bytesOf(outp).buffer, bytesOf(outp).byteOffset, 1)[0] = Deno.fakeCpuShare || 16;
    return 0;
  },
  // tv_verify: the host's availability bits (shard-relative) and, unless Deno.fakeAvailOnly (the files plan
  // check), the SHA-1 of every staged piece against its digest
  tv_verify(ctx, availp, outp) {
    const c = contexts.get(ctx);
    const out = bytesOf(outp);
    const n = Math.ceil(c.count / 8);
    if (availp === null) out.fill(0xff, 0, n);
    else out.set(bytesOf(availp).subarray(0, n));
    if (Deno.fakeAvailOnly) return 0;
    for (let j = 0; j < c.count; j++) {
      const i = c.first + j;
      const d = c.digests.slice(20 * i, 20 * i + 20);
      const data = c.staged.get(i);
      const ok = data && d.length === 20 && crypto.createHash("sha1").update(data).digest().equals(d);
      if (!ok) out[j >> 3] &= ~(0x80 >> (j % 8));
    }
    return 0;
  },
  // tv_hash: the SHA-1 of every staged shard piece (an unstaged piece hashes as its zero bytes)
  tv_hash(ctx, outp) {
    const c = contexts.get(ctx);
    const out = bytesOf(outp);
    for (let j = 0; j < c.count; j++) {
      const i = c.first + j;
      const plen = i === c.P - 1 && c.total % c.L ? c.total % c.L : c.L;
      out.set(crypto.createHash("sha1").update(c.staged.get(i) || Buffer.alloc(plen)).digest(), 20 * j);
    }
    return 0;
  },
  tv_destroy(ctx) {
    // the real library must not be destroyed beside a call still running on another thread
    const c = contexts.get(ctx);
    if (c && c.inflight > 0) Deno.fakeViolations.push("tv_destroy while a nonblocking call runs on the context");
    contexts.delete(ctx);
  },
  tv_last_error: () => 0,
};

const Deno = {
  dlopen(_path, symbols) {
    api.checkSymbols(symbols);
    const out = {};
    for (const name of Object.keys(symbols)) {
      const f = impl[name] || (() => {
        throw new Error(`fake_deno: ${name} is not modelled`);
      });
      out[name] = symbols[name].nonblocking
        ? (...a) => new Promise((res, rej) => {
          const c = name === "tv_create" ? null : contexts.get(a[0]);
          if (c) c.inflight = (c.inflight || 0) + 1;
          const run = () => {
            if (c) c.inflight--;
            try {
              res(f(...a));
            } catch (e) {
              rej(e);
            }
          };
          if (Deno.fakeDelayMs > 0) setTimeout(run, Deno.fakeDelayMs);
          else setImmediate(run);
        })
        : f;
    }
    return { symbols: out, close() {} };
  },
  UnsafePointer: {
    of(ta) {
      const a = nextAddress;
      // (addresses at least one page apart and past the array's end, so an interior pointer names one array)
      nextAddress += (BigInt(ta.byteLength) + 0x1fffn) / 0x1000n * 0x1000n;
      memory.set(a, ta);
      return a;
    },
    create: (v) => (v === 0n ? null : v),
    value: (p) => (p === null ? 0n : p),
  },
  UnsafePointerView: {
    getArrayBuffer(p, len) {
      const ta = memory.get(p);
      if (!ta || ta.byteLength < len) throw new Error("fake_deno: getArrayBuffer of an unknown or short pointer");
      return ta.buffer;
    },
  },
  fakeContexts: contexts,
  fakeDelayMs: 0,
  fakeViolations: [],
  fakeReset() {
    contexts.clear();
    memory.clear();
  },
};

globalThis.Deno = Deno;
if (typeof globalThis.performance === "undefined") globalThis.performance = require("perf_hooks").performance;
module.exports = Deno;
