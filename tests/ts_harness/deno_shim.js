// deno_shim.js -- the Deno globals ts/verify.ts uses, on Node 12 (test infrastructure only; see deno_ffi.cc).
//
//   Deno.dlopen(path, symbols)            symbol table as ts/verify.ts declares it ({parameters, result,
//                                         nonblocking}); "pointer" arguments are BigInt addresses or null,
//                                         "u64" / "usize" / "i64" BigInt, "i32" number.  A nonblocking symbol
//                                         returns a Promise and runs on a libuv worker thread (Deno: its
//                                         blocking-task pool), so calls on different contexts overlap.
//   Deno.UnsafePointer.of / create / value, Deno.UnsafePointerView.getArrayBuffer
//   performance (Node 12 keeps it in perf_hooks)
"use strict";
const path = require("path");
const native = require(path.join(__dirname, "deno_ffi.node"));
const api = require("./deno_api.js");   // the FFI surface of the binding's minimum Deno (1.31)

function arg(kind, v) {
  switch (kind) {
    case "pointer":
      return v === null || v === undefined ? 0n : BigInt.asUintN(64, BigInt(v));
    case "u64":
    case "usize":
    case "i64":
      return BigInt.asUintN(64, BigInt(v));
    case "i32":
      return BigInt.asUintN(64, BigInt(v));
    default:
      throw new Error(`deno_shim: parameter kind ${kind} is not supported`);
  }
}

const Deno = {
  dlopen(file, symbols) {
    api.checkSymbols(symbols);
    const h = native.open(file);
    const out = {};
    for (const name of Object.keys(symbols)) {
      const def = symbols[name];
      const fn = native.sym(h, name);
      const kinds = def.parameters;
      const ret = def.result === "void" ? 0 : def.result === "i32" ? 1 : -1;
      if (ret < 0) throw new Error(`deno_shim: result kind ${def.result} is not supported`);
      const regs = (args) => {
        if (args.length !== kinds.length) throw new Error(`${name}: ${args.length} arguments, ${kinds.length} declared`);
        return kinds.map((k, i) => arg(k, args[i]));
      };
      // a nonblocking symbol runs on a worker thread and resolves later, as Deno's blocking pool does
      out[name] = def.nonblocking
        ? (...args) => {
          try {
            return native.callAsync(fn, regs(args), ret);
          } catch (e) {
            return Promise.reject(e);
          }
        }
        : (...args) => native.call(fn, regs(args), ret);
    }
    return { symbols: out, close() {} };
  },
  UnsafePointer: {
    of(ta) {
      return native.addressOf(ta);
    },
    create(v) {
      return v === 0n ? null : v;
    },
    value(p) {
      return p === null ? 0n : p;
    },
  },
  UnsafePointerView: {
    getArrayBuffer(p, len) {
      return native.arrayBuffer(p, len);
    },
  },
};

globalThis.Deno = Deno;
if (typeof globalThis.performance === "undefined") globalThis.performance = require("perf_hooks").performance;
module.exports = Deno;
