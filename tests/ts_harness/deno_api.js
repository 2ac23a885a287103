// deno_api.js -- the Deno FFI surface ts/verify.ts may use: that of its stated minimum, Deno 1.31 (INTEGRATION.md).
// Test infrastructure only: deno_shim.js (the real library under Node) and fake_deno.js (the CPU model) both check
// every Deno.dlopen symbol table against it, so a binding that starts using an FFI feature newer than 1.31 fails
// on CPU.  What 1.31 has and the binding relies on:
//   Deno.dlopen(path, {name: {parameters, result, nonblocking?}})    (nonblocking since 1.15)
//   parameter / result types as strings: the integer and float kinds, "pointer", "buffer", "function", "void"
//   Deno.UnsafePointer.of / create / value and Deno.PointerValue = null | pointer object (1.31: pointers became
//   objects; UnsafePointer.create / value replaced bigint pointers), Deno.UnsafePointerView.getArrayBuffer
// Newer and therefore rejected: struct types ({struct: [...]}, 1.35), `optional` symbols (1.36), "bool" (1.3x).
"use strict";
const MIN_VERSION = "1.31";
const TYPES = new Set(["i8", "u8", "i16", "u16", "i32", "u32", "i64", "u64", "usize", "isize", "f32", "f64",
                       "pointer", "buffer", "function"]);
const KEYS = new Set(["parameters", "result", "nonblocking"]);

function checkSymbols(symbols) {
  for (const [name, def] of Object.entries(symbols)) {
    for (const k of Object.keys(def)) {
      if (!KEYS.has(k)) throw new Error(`deno_api: ${name}: symbol option "${k}" needs a Deno newer than ${MIN_VERSION}`);
    }
    for (const t of def.parameters) {
      if (typeof t !== "string" || !TYPES.has(t)) {
        throw new Error(`deno_api: ${name}: parameter type ${JSON.stringify(t)} needs a Deno newer than ${MIN_VERSION}`);
      }
    }
    if (typeof def.result !== "string" || !(TYPES.has(def.result) || def.result === "void")) {
      throw new Error(`deno_api: ${name}: result type ${JSON.stringify(def.result)} needs a Deno newer than ${MIN_VERSION}`);
    }
  }
}

// the Deno namespace members (and their members) a 1.31 runtime provides that the harness models
const SURFACE = ["dlopen", "UnsafePointer.of", "UnsafePointer.create", "UnsafePointer.value",
                 "UnsafePointerView.getArrayBuffer", "PointerValue", "DynamicLibrary"];

module.exports = { MIN_VERSION, checkSymbols, SURFACE };
