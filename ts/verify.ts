// ts/verify.ts -- Deno binding of libtorrent_verify.so: the new verify module for rclarey/torrent.
//
// Drop-in position: next to piece.ts / storage.ts in the reference.  It imports only the
// reference's own types (InfoDict from metainfo.ts:12-44, Storage from storage.ts:34-138,
// pieceLength rule of piece.ts:16-19) and replaces nothing: callers of Storage / InfoDict /
// Torrent are unaffected.  The SHA-1 arithmetic that the reference runs through
// crypto.subtle.digest("SHA-1", content) (tools/make_torrent.ts:28-31) runs on the GPU here.
//
// Requires: Deno 1.31 or newer (the pointer-object FFI: Deno.UnsafePointer.create / .value and Deno.PointerValue
// objects; `nonblocking` symbols, 1.15), run as deno run --unstable --allow-ffi (Deno 1.x, as the reference CI:
// .github/workflows/main.yml:13-14, deno-version v1.x).  tests/ts_harness/deno_api.js holds that version's FFI
// surface, and both harness shims reject a symbol table that goes beyond it.
// Deno is not installed in the build container: tests/test_ts_binding.py runs this file under Node 12 with an
// N-API shim of Deno's FFI on the GPU (tests/ts_harness/deno_shim.js) and against a JS model of the library
// on CPU (tests/ts_harness/fake_deno.js).

import type { InfoDict } from "../metainfo.ts";
import type { Storage } from "../storage.ts";

const SYMBOLS = {
  tv_abi_version: { parameters: [], result: "i32" },
  tv_device_count: { parameters: ["pointer"], result: "i32" },
  tv_cpu_share: { parameters: ["pointer"], result: "i32" },
  tv_create: { parameters: ["pointer", "i32"], result: "i32" },
  tv_destroy: { parameters: ["pointer"], result: "void" },
  tv_last_error: { parameters: ["pointer", "pointer", "usize"], result: "i32" },
  tv_set_layout: { parameters: ["pointer", "u64", "u64", "u64", "u64", "u64"], result: "i32" },
  tv_set_digests: { parameters: ["pointer", "pointer", "u64"], result: "i32" },
  tv_stage: { parameters: ["pointer", "u64", "pointer", "u64"], result: "i32", nonblocking: true },
  tv_stage_many: { parameters: ["pointer", "u64", "pointer", "pointer", "pointer"], result: "i32", nonblocking: true },
  tv_stage_file: { parameters: ["pointer", "pointer", "u64", "u64", "u64"], result: "i32", nonblocking: true },
  tv_stage_files: {
    parameters: ["pointer", "u64", "pointer", "pointer", "pointer", "pointer", "pointer"],
    result: "i32",
    nonblocking: true,
  },
  tv_stage_file_table: {
    parameters: ["pointer", "u64", "pointer", "pointer", "u64", "pointer"],
    result: "i32",
    nonblocking: true,
  },
  tv_stream_file_table: {
    parameters: ["pointer", "u64", "pointer", "pointer", "u64", "pointer", "pointer", "pointer"],
    result: "i32",
    nonblocking: true,
  },
  tv_read: { parameters: ["pointer", "u64", "pointer", "u64"], result: "i32", nonblocking: true },
  tv_fill_synthetic: { parameters: ["pointer", "u64"], result: "i32" },
  tv_verify: { parameters: ["pointer", "pointer", "pointer"], result: "i32", nonblocking: true },
  tv_verify_host: {
    parameters: ["pointer", "pointer", "u64", "pointer", "pointer"],
    result: "i32",
    nonblocking: true,
  },
  tv_verify_list: { parameters: ["pointer", "pointer", "u64", "pointer"], result: "i32", nonblocking: true },
  tv_hash: { parameters: ["pointer", "pointer"], result: "i32", nonblocking: true },
  tv_stream_begin: { parameters: ["pointer", "pointer"], result: "i32" },
  tv_stream_next: { parameters: ["pointer", "pointer"], result: "i32", nonblocking: true },
  tv_stream_commit: { parameters: ["pointer", "pointer"], result: "i32", nonblocking: true },
  tv_stream_commit_from: { parameters: ["pointer", "pointer", "pointer", "u64"], result: "i32", nonblocking: true },
  tv_stream_unreadable: { parameters: ["pointer", "u64"], result: "i32" },
  tv_stream_end: { parameters: ["pointer", "pointer"], result: "i32", nonblocking: true },
  tv_stream_abort: { parameters: ["pointer"], result: "i32" },
  tv_stream_fill_synthetic: { parameters: ["pointer", "pointer", "u64"], result: "i32", nonblocking: true },
  tv_set_option: { parameters: ["pointer", "i32", "i64"], result: "i32" },
  tv_get_option: { parameters: ["pointer", "i32", "pointer"], result: "i32" },
  tv_last_timing: { parameters: ["pointer", "pointer", "pointer"], result: "i32" },
  tv_last_kernel: { parameters: ["pointer", "pointer", "pointer"], result: "i32" },
  tv_get_counter: { parameters: ["pointer", "i32", "pointer"], result: "i32" },
  tv_synchronize: { parameters: ["pointer"], result: "i32" },
  tv_host_alloc: { parameters: ["u64", "pointer"], result: "i32" },
  tv_host_free: { parameters: ["pointer"], result: "i32" },
  tv_host_register: { parameters: ["pointer", "u64"], result: "i32" },
  tv_host_unregister: { parameters: ["pointer"], result: "i32" },
} as const;

export interface VerifyOptions {
  /** path of libtorrent_verify.so (default: ./torrent_amd/libtorrent_verify.so) */
  libPath?: string;
  /** GPU indices; pieces are sharded over them in contiguous, 8-aligned ranges */
  devices?: number[];
  /** pieces read through storage.get per staging batch */
  batchBytes?: number;
  /** bytes of device memory the payload may take per device (default: the GPU's free memory less a margin); a
   * shard larger than it is verified in windows of pieces that fit, each hashed while the next one stages */
  budget?: number;
  /** verifyPiece only: hash on the CPU with the reference's own crypto.subtle.digest("SHA-1", bytes)
   * (tools/make_torrent.ts:28-31) instead of a ~3 ms GPU launch.  Off by default */
  cpuFallback?: boolean;
  /** verifyFiles: read the shard's files through the bounded ring in columns within `budget` (tv_stream_file_table:
   * the library picks windows of >= 2,048 pieces and columns as wide as the budget allows) instead of holding
   * windows of whole pieces in device memory -- the faster form under a small budget, where each window pays one
   * piece's serial SHA-1 (default: chosen per shard, streamWins) */
  stream?: boolean;
  /** host threads the library may use for one call, over all of its shards (default: the process's CPU share as
   * the library reads it, tv_cpu_share: the cgroup quota, else OMP_NUM_THREADS, else the affinity mask): each
   * shard's context gets its part (TV_OPT_FILE_THREADS), so devices [0..7] do not start 8 x 16 reader threads */
  threads?: number;
}

const TV_OPT_FILE_THREADS = 8;

/** The process's CPU share as the library reads it (tv_cpu_share; cached).  The library reads the cgroup files
 * itself, so a Deno process without --allow-read still gets the container's quota, not the machine's cores. */
let cpuShareCache = 0;
function libCpuShare(l: Lib | null): number {
  if (!cpuShareCache && l) {
    const out = new Uint32Array(1);
    if (l.symbols.tv_cpu_share(ptr(new Uint8Array(out.buffer))) === 0) cpuShareCache = out[0];
  }
  return cpuShareCache;
}

/** Reader / copy threads of each of `active` concurrently running shards: opts.threads (else the process's CPU
 * share, tv_cpu_share) divided among them, 1 .. 16 each (16 is the library's default; its page-cache readers
 * already saturate PCIe there).  Same rule as torrent_amd/_cpu.py shard_threads, without its per-NUMA-node cap. */
export function shardThreads(opts: VerifyOptions, active: number, l: Lib | null = lib): number {
  const share = opts.threads || libCpuShare(l) ||
    (typeof navigator !== "undefined" && navigator.hardwareConcurrency) || 16;
  return Math.max(1, Math.min(16, Math.floor(share / Math.max(1, active))));
}

function activeShards(ranges: [number, number][]): number {
  return ranges.filter(([, count]) => count > 0).length;
}

/** SHA-1(bytes) === digest through WebCrypto, the reference's SHA-1 path (make_torrent.ts:28-31). */
async function cpuPieceOk(bytes: Uint8Array, digest: Uint8Array): Promise<boolean> {
  if (digest.length !== 20) return false;
  const d = new Uint8Array(await crypto.subtle.digest("SHA-1", bytes));
  for (let k = 0; k < 20; k++) if (d[k] !== digest[k]) return false;
  return true;
}

const TV_OPT_RESIDENT_BUDGET = 16;
const TV_OPT_LIST_SLOTS = 17;

type Lib = Deno.DynamicLibrary<typeof SYMBOLS>;
let lib: Lib | null = null;

function load(path?: string): Lib {
  if (!lib) {
    lib = Deno.dlopen(path === undefined ? "./torrent_amd/libtorrent_verify.so" : path, SYMBOLS);
    if (lib.symbols.tv_abi_version() !== 1) throw new Error("libtorrent_verify ABI mismatch");
  }
  return lib;
}

function ptr(a: Uint8Array | null): Deno.PointerValue {
  return a ? Deno.UnsafePointer.of(a) : null;
}

function check(l: Lib, ctx: Deno.PointerValue, rc: number): void {
  if (rc !== 0) {
    const buf = new Uint8Array(1024);
    const n = l.symbols.tv_last_error(ctx, ptr(buf), BigInt(buf.length));
    throw new Error(`torrent_verify error ${rc}: ${new TextDecoder().decode(buf.subarray(0, Math.min(n, 1023)))}`);
  }
}

/**
 * One cached context per (device, shard slot), held exclusively for a whole job: device memory and the
 * pinned staging ring are reused across calls (tv_set_layout keeps allocations that fit), so a
 * verifyPiece does not pay tv_create + stream/event creation + a 192 MiB pinned ring each time.  Jobs on
 * one context take turns (a promise chain), so a job's set_layout -> stage -> verify sequence is never
 * interleaved with another's.  Same policy as torrent_amd/verify.py _context.
 */
const contexts = new Map<string, { ctx: Deno.PointerValue; tail: Promise<void> }>();

async function withContext<T>(l: Lib, device: number, slot: number, job: (ctx: Deno.PointerValue) => Promise<T>): Promise<T> {
  const key = `${device}:${slot}`;
  let e = contexts.get(key);
  if (!e) {
    const h = new BigUint64Array(1);
    check(l, null, l.symbols.tv_create(ptr(new Uint8Array(h.buffer)), device));
    e = { ctx: Deno.UnsafePointer.create(h[0]), tail: Promise.resolve() };
    contexts.set(key, e);
  }
  const entry = e;
  const run = entry.tail.then(() => job(entry.ctx));
  entry.tail = run.then(() => {}, () => {});
  return await run;
}

/** tv_set_layout under this call's device budget (contexts are cached: every call sets its own). */
function setLayout(l: Lib, ctx: Deno.PointerValue, total: number, L: number, P: number, first: number, count: number,
                   budget?: number): void {
  check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT_BUDGET, BigInt(budget || 0)));
  check(l, ctx, l.symbols.tv_set_layout(ctx, BigInt(total), BigInt(L), BigInt(P), BigInt(first), BigInt(count)));
}

/** Free every cached context (device payload, pinned ring); the next call creates new ones. */
export async function releaseContexts(): Promise<void> {
  const all = [...contexts.values()];
  contexts.clear();
  for (const e of all) {
    await e.tail;
    if (lib) lib.symbols.tv_destroy(e.ctx);
  }
}

/** piece.ts:16-19 (private there; restated) */
function pieceLength(n: number, info: InfoDict): number {
  return (n === info.pieces.length - 1 && info.length % info.pieceLength) || info.pieceLength;
}

/** contiguous shards of whole bitfield bytes (first % 8 === 0) */
export function shardRanges(nPieces: number, nShards: number): [number, number][] {
  const per = Math.ceil(Math.ceil(nPieces / nShards) / 8) * 8;
  const out: [number, number][] = [];
  for (let s = 0, first = 0; s < nShards; s++) {
    const count = Math.max(0, Math.min(per, nPieces - first));
    out.push([first, count]);
    first += count;
  }
  return out;
}

function piecesRaw(info: InfoDict): Uint8Array {
  // metainfo.ts:111 partition() returns contiguous views of the .torrent buffer; rebuild the string
  const total = info.pieces.reduce((n, p) => n + p.length, 0);
  const out = new Uint8Array(total);
  let o = 0;
  for (const p of info.pieces) {
    out.set(p, o);
    o += p.length;
  }
  return out;
}

/** storage.get calls a bulk verify keeps outstanding (file descriptors, not bandwidth, bound it) */
const READS_IN_FLIGHT = 32;

/** fn(0..n-1), at most READS_IN_FLIGHT of them pending at a time. */
async function eachLimited(n: number, fn: (q: number) => Promise<void>): Promise<void> {
  let next = 0;
  const worker = async () => {
    for (let q = next++; q < n; q = next++) await fn(q);
  };
  await Promise.all(Array.from({ length: Math.min(READS_IN_FLIGHT, n) }, worker));
}

/**
 * verifyPieces(info, storage) -> have-bitfield (Uint8Array of ceil(P/8) bytes, MSB-first:
 * torrent.ts:53,60,147-149).  Piece i's bit is set iff storage.get(i*pieceLength, len_i) is
 * non-null (storage.ts:50-65) and its SHA-1 equals info.pieces[i].  Unreadable pieces are 0, not
 * errors (the reference swallows I/O failures into null); GPU / ABI failures throw Error.  Reads and
 * staging overlap: batch k + 1 is read while batch k's pieces -- the Uint8Arrays storage.get returned, never
 * gathered on this thread -- are copied into the library's pinned ring and DMA'd (tv_stage_many, nonblocking).
 */
export async function verifyPieces(
  info: InfoDict,
  storage: Storage,
  opts: VerifyOptions = {},
): Promise<Uint8Array> {
  const l = load(opts.libPath);
  const P = info.pieces.length;
  const L = info.pieceLength;
  const devices = opts.devices || [0];
  const raw = piecesRaw(info);
  const bitfield = new Uint8Array(Math.ceil(P / 8));
  const batch = Math.max(1, Math.floor((opts.batchBytes || 256 * 2 ** 20) / L));

  const ranges = shardRanges(P, devices.length);
  const threads = shardThreads(opts, activeShards(ranges));
  await Promise.all(ranges.map(async ([first, count], s) => {
    if (count === 0) return;
    await withContext(l, devices[s], s, async (ctx) => {
      setLayout(l, ctx, info.length, L, P, first, count, opts.budget);
      // tv_stage_many copies the batch's buffers into the pinned ring on this many library threads
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_FILE_THREADS, BigInt(threads)));
      check(l, ctx, l.symbols.tv_set_digests(ctx, ptr(raw), BigInt(raw.length)));
      const avail = new Uint8Array(Math.ceil(count / 8));
      const per = Math.min(batch, count);
      const u8 = (a: ArrayBufferView) => new Uint8Array(a.buffer, a.byteOffset, a.byteLength);
      let staging: Promise<void> | null = null; // the previous batch's tv_stage_many (it still reads its buffers)
      try {
        for (let j = 0; j < count; j += per) {
          const k = Math.min(per, count - j);
          const got: (Uint8Array | null)[] = new Array(k).fill(null);
          // READS_IN_FLIGHT reads outstanding at a time (make_torrent.ts:96,111 keeps its work in flight too, but
          // each fsStorage.get is a Deno.open: a batch of 16 KiB pieces at once would hit EMFILE, which
          // fsStorage.get turns into null -- a valid piece reported 0)
          await eachLimited(k, async (q) => {
            const n = pieceLength(first + j + q, info);
            const bytes = await storage.get((first + j + q) * L, n);
            // Storage.get returns exactly the length asked or null; any other length is unreadable too (as in
            // verifyStream)
            if (!bytes || bytes.length !== n) return;
            got[q] = bytes;
            avail[(j + q) >> 3] |= 128 >> ((j + q) % 8);
          });
          if (staging) await staging;
          staging = null;
          // the batch's readable pieces, ascending, handed over as they are: the library copies them into its
          // pinned ring on its own threads (tv_stage_many), so this thread does no gather copy
          const qs = got.map((b, q) => (b ? q : -1)).filter((q) => q >= 0);
          if (qs.length) {
            const offs = new BigUint64Array(qs.length), srcs = new BigUint64Array(qs.length);
            const lens = new BigUint64Array(qs.length);
            qs.forEach((q, t) => {
              const b = got[q] as Uint8Array;
              offs[t] = BigInt((first + j + q) * L);
              srcs[t] = BigInt(Deno.UnsafePointer.value(Deno.UnsafePointer.of(b)));
              lens[t] = BigInt(b.length);
            });
            const keep = [got, offs, srcs, lens]; // alive until the library has read them
            staging = l.symbols.tv_stage_many(ctx, BigInt(qs.length), ptr(u8(offs)), ptr(u8(srcs)), ptr(u8(lens)))
              .then((rc) => {
                keep.length = 0;
                check(l, ctx, rc);
              });
          }
        }
      } finally {
        if (staging) await staging;
      }
      const out = new Uint8Array(Math.ceil(count / 8));
      check(l, ctx, await l.symbols.tv_verify(ctx, ptr(avail), ptr(out)));
      bitfield.set(out, first / 8);
    });
  }));
  return bitfield;
}

const TV_OPT_STREAM_CHUNK = 3;
const TV_OPT_RESIDENT = 10;
const TV_OPT_OPEN_RW = 18;
const TV_OPT_STREAM_ROWS = 19;

/**
 * verifyStream(info, storage) -> have-bitfield: the end-to-end resume check through the library's
 * BOUNDED pinned ring (tv_stream_*; SURVEY 8d config 5; the resume flow Client.add -> verify ->
 * Torrent.bitfield -> sendBitfield, client.ts:53-67, torrent.ts:56-60,101).  No resident payload and no
 * whole-shard buffer: the library requests the shard in rows of whole pieces (TV_OPT_STREAM_ROWS; with
 * opts.chunk, column by column: bytes [c*C, c*C + C) of every piece), each row is one
 * storage.get(offset, length) written straight into the library's pinned slot -- one fsStorage open per
 * piece -- and the library DMAs the slot to HBM while the GPU hashes the previous window.  Host memory in flight:
 * 3 x 64 MiB per device.  null from storage.get makes that piece 0 (a piece is readable iff every slice
 * of it reads).  Same behaviour as torrent_amd.verify_stream.
 */
export async function verifyStream(info: InfoDict, storage: Storage, opts: VerifyOptions & { chunk?: number } = {}): Promise<Uint8Array> {
  const l = load(opts.libPath);
  const P = info.pieces.length;
  const L = info.pieceLength;
  const devices = opts.devices || [0];
  const raw = piecesRaw(info);
  const bitfield = new Uint8Array(Math.ceil(P / 8));
  const ranges = shardRanges(P, devices.length);
  const threads = shardThreads(opts, activeShards(ranges));
  await Promise.all(ranges.map(async ([first, count], s) => {
    if (count === 0) return;
    await withContext(l, devices[s], s, async (ctx) => {
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT, 0n));
      // (a budget an earlier call left on the cached context would cap the row windows)
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT_BUDGET, 0n));
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_FILE_THREADS, BigInt(threads)));
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_STREAM_CHUNK, BigInt(opts.chunk || 0)));
      // default: whole pieces per row (one storage.get, i.e. one fsStorage open, per piece); chunk: columns
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_STREAM_ROWS, opts.chunk ? 0n : 1n));
      try {
        check(l, ctx, l.symbols.tv_set_layout(ctx, BigInt(info.length), BigInt(L), BigInt(P), BigInt(first), BigInt(count)));
      } finally {
        l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT, 1n);
      }
      check(l, ctx, l.symbols.tv_set_digests(ctx, ptr(raw), BigInt(raw.length)));
      check(l, ctx, l.symbols.tv_stream_begin(ctx, null));
      const req = new BigUint64Array(6); // tv_stream_req: piece, rows, offset, width, slot, seq
      const reqp = ptr(new Uint8Array(req.buffer));
      try {
        for (;;) {
          check(l, ctx, await l.symbols.tv_stream_next(ctx, reqp));
          const rows = Number(req[1]);
          if (rows === 0) break;
          const piece = Number(req[0]), offset = Number(req[2]), width = Number(req[3]);
          const slot = new Uint8Array(Deno.UnsafePointerView.getArrayBuffer(Deno.UnsafePointer.create(req[4])!, rows * width));
          // READS_IN_FLIGHT reads of the request outstanding at a time: each fsStorage.get is a Deno.open, and
          // an EMFILE from a thousand opens at once would come back as null -- a valid piece reported 0
          await eachLimited(rows, async (q) => {
            const n = Math.max(0, Math.min(width, pieceLength(piece + q, info) - offset));
            if (n === 0) return;
            const bytes = await storage.get((piece + q) * L + offset, n);
            // a row must be exactly n bytes: more would spill into the next row (Python: unreadable too)
            if (bytes && bytes.length === n) slot.set(bytes, q * width);
            else check(l, ctx, l.symbols.tv_stream_unreadable(ctx, BigInt(piece + q)));
          });
          check(l, ctx, await l.symbols.tv_stream_commit(ctx, reqp));
        }
        const out = new Uint8Array(Math.ceil(count / 8));
        check(l, ctx, await l.symbols.tv_stream_end(ctx, ptr(out)));
        bitfield.set(out, first / 8);
      } catch (err) {
        l.symbols.tv_stream_abort(ctx);
        throw err;
      } finally {
        l.symbols.tv_set_option(ctx, TV_OPT_STREAM_CHUNK, 0n);
        l.symbols.tv_set_option(ctx, TV_OPT_STREAM_ROWS, 0n);
      }
    });
  }));
  return bitfield;
}

/**
 * verifyFiles(info, dir) -> have-bitfield of the files under `dir` (resume from disk, SURVEY 8f
 * row f2), laid out as new Storage(fsStorage, info, dir) maps them (storage.ts:89-137: single-file
 * [dir, name], multi-file [dir, ...path]).  Each shard hands the library the torrent's FILE TABLE in one
 * tv_stage_file_table call and the library makes Storage.get's walk itself (the segments of the shard, the
 * zero-length ones fsStorage.get still opens included): long segments are cut into 256 MiB units read by
 * parallel preads into the library's pinned ring on its two staging lanes and DMA'd from there; short ones
 * (many small files) are read by the library's thread pool into pinned slots.  The table (lengths and one
 * NUL-separated path buffer) is built once per (info, dir) and kept, so a repeat call does no per-file encoding.
 * The shard's reader threads are its part of opts.threads (shardThreads).
 * The library marks the pieces fsStorage.get would return null for (storage.ts:163-171): a byte in a
 * missing, unopenable or unwritable file or past a short file's end, or a zero-length segment whose open
 * would fail (a directory, a missing parent directory); unlike fsStorage.get, no missing file is created.  Same
 * behaviour as torrent_amd.verify_files.
 */
/** Numbers (< 2^52) as the little-endian u64 words of a C array (Deno runs on little-endian hosts only), written
 * as 32-bit halves -- a BigInt per element cost ~3-4 ms on a 10,000-file verifyFiles. */
function u64Words(vals: number[]): Uint32Array {
  const out = new Uint32Array(2 * vals.length);
  for (let k = 0; k < vals.length; k++) {
    const hi = Math.floor(vals[k] / 4294967296);
    out[2 * k] = vals[k] - hi * 4294967296;
    out[2 * k + 1] = hi;
  }
  return out;
}

/** A torrent's file table as tv_stage_file_table takes it: file k's length (u64 words) and its path, the k-th
 * NUL-terminated string of one buffer.  A path holding a NUL cannot be opened (Deno.open refuses it, so
 * fsStorage.get's piece is null): it goes as "", which the library cannot open either. */
interface FileTable {
  dir: string;
  n: number;
  lengths: Uint32Array;
  paths: Uint8Array;
  // what it was built from: each file's length and path (array) object, compared on reuse without allocating
  lens: number[];
  refs: (string[] | string)[];
}
const fileTables = new WeakMap<InfoDict, FileTable>();

function fileTable(info: InfoDict, dir: string): FileTable {
  const files = "files" in info ? info.files : null;
  const n = files ? files.length : 1;
  const lenOf = (k: number) => files ? files[k].length : info.length;
  const refOf = (k: number): string[] | string => files ? files[k].path : info.name;
  const hit = fileTables.get(info);
  if (hit && hit.dir === dir && hit.n === n) {
    let same = true;
    for (let k = 0; k < n && same; k++) same = hit.lens[k] === lenOf(k) && hit.refs[k] === refOf(k);
    if (same) return hit;
  }
  const enc = new TextEncoder();
  const lens: number[] = [];
  const refs: (string[] | string)[] = [];
  const joined: string[] = [];
  for (let k = 0; k < n; k++) {
    const r = refOf(k);
    lens.push(lenOf(k));
    refs.push(r);
    joined.push(typeof r === "string" ? [dir, r].join("/") : [dir, ...r].join("/"));
  }
  let cap = n;
  for (const p of joined) cap += 3 * p.length;   // (UTF-8: at most 3 bytes per UTF-16 code unit)
  const buf = new Uint8Array(cap);
  let o = 0;
  for (const p of joined) {
    if (!p.includes("\0")) o += enc.encodeInto(p, buf.subarray(o)).written;
    buf[o++] = 0;
  }
  const t = { dir, n, lengths: u64Words(lens), paths: buf.subarray(0, o), lens, refs };
  fileTables.set(info, t);
  return t;
}

/** Whether a file-backed shard verifies faster in streamed columns than in windows of whole pieces under the device
 * budget (torrent_amd/verify.py _stream_wins): the shard does not fit it, and windows would cost more than staging
 * (each pays one piece's serial SHA-1, ~11.8 ms per MiB of piece: below ~0.9 GB of budget per MiB of piece length). */
export function streamWins(L: number, count: number, budget?: number): boolean {
  if (!budget) return false;
  const stride = Math.ceil(L / 64) * 64 + 256;
  return count * stride + 256 > budget && budget < 0.9e9 * L / 1048576;
}

export async function verifyFiles(info: InfoDict, dir: string, opts: VerifyOptions = {}): Promise<Uint8Array> {
  const l = load(opts.libPath);
  const P = info.pieces.length;
  const L = info.pieceLength;
  const devices = opts.devices || [0];
  const raw = piecesRaw(info);
  const table = fileTable(info, dir);
  const bitfield = new Uint8Array(Math.ceil(P / 8));
  const u8 = (a: ArrayBufferView) => new Uint8Array(a.buffer, a.byteOffset, a.byteLength);

  const ranges = shardRanges(P, devices.length);
  const threads = shardThreads(opts, activeShards(ranges), l);
  await Promise.all(ranges.map(async ([first, count], s) => {
    if (count === 0) return;
    await withContext(l, devices[s], s, async (ctx) => {
      if (opts.stream || (opts.stream === undefined && streamWins(L, count, opts.budget))) {
        // columns through the bounded ring, read by the library from the file table
        check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT, 0n));
        // (the library sizes windows x columns to the budget)
        check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT_BUDGET, BigInt(opts.budget || 0)));
        check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_STREAM_CHUNK, 0n));
        check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_STREAM_ROWS, 0n));
        try {
          check(l, ctx, l.symbols.tv_set_layout(ctx, BigInt(info.length), BigInt(L), BigInt(P), BigInt(first),
                                                BigInt(count)));
        } finally {
          l.symbols.tv_set_option(ctx, TV_OPT_RESIDENT, 1n);
        }
        check(l, ctx, l.symbols.tv_set_digests(ctx, ptr(raw), BigInt(raw.length)));
        check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_OPEN_RW, 1n));
        check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_FILE_THREADS, BigInt(threads)));
        const status = new Int32Array(table.n);
        const out = new Uint8Array(Math.ceil(count / 8));
        check(l, ctx, await l.symbols.tv_stream_file_table(ctx, BigInt(table.n), ptr(u8(table.lengths)),
                                                           ptr(table.paths), BigInt(table.paths.length), null,
                                                           ptr(out), ptr(u8(status))));
        bitfield.set(out, first / 8);
        return;
      }
      setLayout(l, ctx, info.length, L, P, first, count, opts.budget);
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_OPEN_RW, 1n)); // fsStorage.get's read + write open
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_FILE_THREADS, BigInt(threads))); // this shard's readers
      check(l, ctx, l.symbols.tv_set_digests(ctx, ptr(raw), BigInt(raw.length)));
      const avail = new Uint8Array(Math.ceil(count / 8)).fill(0xff);
      if (count % 8) avail[avail.length - 1] = (0xff00 >> (count % 8)) & 0xff;
      // pieces whose bytes extend past the last file (more digests than data) are unreadable
      for (let j = count - 1; j >= 0 && (first + j) * L + pieceLength(first + j, info) > info.length; j--) {
        avail[j >> 3] &= ~(128 >> (j % 8));
      }
      // the shard's segments of findAndDo's walk (storage.ts:105-128), made by the library from the table; a failed
      // segment's pieces are marked inside the library (tv_verify reports them 0), from the piece holding its first
      // unreadable byte on, as Storage.get reads piece by piece: the per-file `status` is informational
      const status = new Int32Array(table.n);
      check(l, ctx, await l.symbols.tv_stage_file_table(ctx, BigInt(table.n), ptr(u8(table.lengths)), ptr(table.paths),
                                                        BigInt(table.paths.length), ptr(u8(status))));
      const out = new Uint8Array(Math.ceil(count / 8));
      check(l, ctx, await l.symbols.tv_verify(ctx, ptr(avail), ptr(out)));
      bitfield.set(out, first / 8);
    });
  }));
  return bitfield;
}

/** verifyPiece(info, index, bytes): one piece (e.g. on completion of its last 16 KiB block). */
export async function verifyPiece(info: InfoDict, index: number, bytes: Uint8Array, opts: VerifyOptions = {}): Promise<boolean> {
  // piece.ts:22 rejects index >= pieces.length; a negative or fractional index is no piece either (as verify.py)
  if (!Number.isInteger(index) || index < 0 || index >= info.pieces.length) {
    throw new Error(`verifyPiece: invalid piece index ${index}`);
  }
  if (bytes.length !== pieceLength(index, info) || info.pieces[index].length !== 20) return false;
  if (opts.cpuFallback) return await cpuPieceOk(bytes, info.pieces[index]);
  const l = load(opts.libPath);
  // its own cached context (slot -1): a one-piece layout on a bulk call's context would free that context's
  // payload (tv_set_layout keeps an allocation only while the new geometry is at least half of it)
  return await withContext(l, (opts.devices || [0])[0], -1, async (ctx) => {
    const n = BigInt(bytes.length);
    setLayout(l, ctx, bytes.length, bytes.length, 1, 0, 1); // reuses the context's allocations
    check(l, ctx, l.symbols.tv_set_digests(ctx, ptr(info.pieces[index]), 20n));
    check(l, ctx, await l.symbols.tv_stage(ctx, 0n, ptr(bytes), n));
    const out = new Uint8Array(1);
    check(l, ctx, await l.symbols.tv_verify(ctx, null, ptr(out)));
    return (out[0] & 0x80) !== 0;
  });
}

/**
 * hashPieces(payload, pieceLength) -> the `pieces` string (20 B per piece) of a linear payload:
 * creation mode (SURVEY 8f row f3), the GPU form of make_torrent.ts:147-173 (single file) and
 * :62-113 (files concatenated in order).  Pieces are sharded over `opts.devices` as verifyPieces shards
 * them; each shard's digests land at 20 * first.  Same behaviour as torrent_amd.hash_pieces.
 */
export async function hashPieces(payload: Uint8Array, pieceLength: number, opts: VerifyOptions = {}): Promise<Uint8Array> {
  const P = Math.ceil(payload.length / pieceLength);
  if (P === 0) return new Uint8Array(0);
  const l = load(opts.libPath);
  const devices = opts.devices || [0];
  const out = new Uint8Array(20 * P);
  const ranges = shardRanges(P, devices.length);
  const threads = shardThreads(opts, activeShards(ranges));
  await Promise.all(ranges.map(async ([first, count], s) => {
    if (count === 0) return;
    await withContext(l, devices[s], s, async (ctx) => {
      setLayout(l, ctx, payload.length, pieceLength, P, first, count, opts.budget);
      check(l, ctx, l.symbols.tv_set_option(ctx, TV_OPT_FILE_THREADS, BigInt(threads)));
      const lo = first * pieceLength, hi = Math.min(payload.length, (first + count) * pieceLength);
      if (hi > lo) check(l, ctx, await l.symbols.tv_stage(ctx, BigInt(lo), ptr(payload.subarray(lo, hi)), BigInt(hi - lo)));
      const digests = new Uint8Array(20 * count);
      check(l, ctx, await l.symbols.tv_hash(ctx, ptr(digests)));
      out.set(digests, 20 * first);
    });
  }));
  return out;
}

/** Options of PieceVerifier's flush policy (same defaults as torrent_amd/incremental.py). */
export interface FlushPolicy {
  /** flush once this many completed pieces are pending (default 4,096: a flush's time is flat up to there) */
  flushPieces?: number | null;
  /** flush once the oldest pending piece is this old (default 10 x the flush cost, >= 5 ms: ~30 ms at 256 KiB) */
  flushAgeMs?: number | null;
  /** results of automatic flushes (else they are returned by the next flush()) */
  onVerified?: (index: number, ok: boolean) => void;
  /** flushes of at most this many pieces are hashed on the CPU with crypto.subtle.digest (the reference's SHA-1,
   * make_torrent.ts:28-31) instead of one GPU list launch; completed pieces then wait host-side and are staged
   * at the flush that goes to the GPU.  0 (default) = off.  The crossover (a GPU flush costs ~one piece's serial
   * SHA-1 whatever the count, 3.0 ms at 256 KiB; a CPU core hashes 256 KiB in 0.2 ms with SHA-NI) is measured
   * by tools/cpu_crossover.py (profiles/r04/cpu_crossover.json) */
  cpuFallbackMaxPieces?: number;
}

/** GPU time of one list flush of pieces of `pieceLength` bytes: one piece's serial SHA-1, ~0.73 us per 64-B
 * block (3.0 ms for 256 KiB, whether 1 or 4,096 pieces: profiles/r02/latency_twin.json, profiles/r03). */
export function flushCostMs(pieceLength: number): number {
  return (Math.floor((pieceLength + 8) / 64) + 1) * 0.73e-3 + 0.06;
}

/**
 * Incremental verification on piece completion (SURVEY 8f row f1), for the MsgId.piece handler
 * (torrent.ts:183-193): onBlock() per received 16 KiB block (after validateReceivedBlock and
 * storage.set); completed pieces are verified in ONE list launch (tv_verify_list) per flush, and their
 * have-bits set (torrent.ts:147-149).  The verifier flushes by itself when flushPieces are pending or the
 * oldest pending piece is flushAgeMs old (a timer is armed when the first piece becomes pending), so a
 * handler never pays a ~3 ms flush per piece.  Device memory is a pool of `slots` pieces (TV_OPT_LIST_SLOTS;
 * default flushPieces, else 4,096) -- the pieces awaiting verification, not the torrent -- and with every slot
 * taken the next completed piece first flushes the pending ones.  `shard` limits the verifier to pieces
 * [first, first + count) (first % 8 === 0) on opts.devices[0], as the Python verifier's shard.  The library
 * calls (stages and flushes) run one at a time in order, so a flush() always returns the results of an
 * automatic flush that was running when it was called.  Same behaviour as torrent_amd/incremental.py.
 */
export class PieceVerifier {
  readonly bitfield: Uint8Array;
  readonly first: number;
  readonly count: number;
  readonly slots: number;
  autoFlushes = 0;
  forcedFlushes = 0;
  #l: Lib;
  #ctx: Deno.PointerValue;
  #bufs = new Map<number, { bytes: Uint8Array; blocks: Set<number> }>();
  #pending: number[] = [];
  #pendingSet = new Set<number>();
  #staging = new Set<number>();
  #oldest = 0;
  #timer: number | undefined;
  #results: [number, boolean][] = [];
  #flushPieces: number | null;
  #flushAgeMs: number | null;
  #onVerified?: (index: number, ok: boolean) => void;
  #busy: Promise<unknown> = Promise.resolve(); // the verifier's library calls, one at a time, in order
  #timerError: unknown = null;   // a timer-driven flush that failed: rethrown by the next call
  #cpuMax: number;               // cpuFallbackMaxPieces
  #held = new Map<number, Uint8Array>();   // (cpuMax > 0) completed pieces' bytes, staged only if the flush is GPU
  #closed = false;

  readonly info: InfoDict;

  constructor(info: InfoDict, opts: VerifyOptions & FlushPolicy & { shard?: [number, number]; slots?: number } = {}) {
    this.info = info;
    this.#l = load(opts.libPath);
    const P = info.pieces.length;
    const [first, count] = opts.shard || [0, P];
    if (!Number.isInteger(first) || !Number.isInteger(count) || first < 0 || count < 0 || first + count > P ||
        (count > 0 && first % 8 !== 0)) {
      throw new Error(`PieceVerifier: invalid shard [${first}, ${first} + ${count}) of ${P} pieces`);
    }
    this.first = first;
    this.count = count;
    this.#flushPieces = opts.flushPieces === undefined ? 4096 : opts.flushPieces;
    this.#flushAgeMs = opts.flushAgeMs === undefined ? Math.max(5, 10 * flushCostMs(info.pieceLength)) : opts.flushAgeMs;
    this.#onVerified = opts.onVerified;
    this.#cpuMax = Math.max(0, Math.floor(opts.cpuFallbackMaxPieces || 0));
    const k = opts.slots !== undefined ? opts.slots : (this.#flushPieces !== null ? this.#flushPieces : 4096);
    this.slots = Math.max(1, Math.min(Math.floor(k), Math.max(1, count)));
    const h = new BigUint64Array(1);
    check(this.#l, null, this.#l.symbols.tv_create(ptr(new Uint8Array(h.buffer)), (opts.devices || [0])[0]));
    this.#ctx = Deno.UnsafePointer.create(h[0]);
    const raw = piecesRaw(info);
    check(this.#l, this.#ctx, this.#l.symbols.tv_set_option(this.#ctx, TV_OPT_LIST_SLOTS, BigInt(this.slots)));
    check(this.#l, this.#ctx, this.#l.symbols.tv_set_layout(this.#ctx, BigInt(info.length), BigInt(info.pieceLength),
                                                            BigInt(P), BigInt(first), BigInt(count)));
    check(this.#l, this.#ctx, this.#l.symbols.tv_set_digests(this.#ctx, ptr(raw), BigInt(raw.length)));
    this.bitfield = new Uint8Array(Math.ceil(P / 8));
  }

  /** `job` after every library call queued before it (stages and flushes run one at a time, in order). */
  private _serial<T>(job: () => Promise<T>): Promise<T> {
    const run = this.#busy.then(job);
    this.#busy = run.catch(() => {});
    return run;
  }

  /** One received block (already validated); true when it completed its piece. */
  async onBlock(index: number, offset: number, block: Uint8Array): Promise<boolean> {
    this._open();
    this._rethrow();
    await this._autoFlush();                                  // the age bound, checked on every block
    if (index < this.first || index >= this.first + this.count) {
      throw new Error(`PieceVerifier: piece ${index} is outside this verifier's shard`);
    }
    if (this.bitfield[index >> 3] & (128 >> (index % 8))) return false;
    if (this.#pendingSet.has(index)) return false; // complete, waiting for a flush: ignore re-sends
    if (this.#staging.has(index)) return false;    // its completing block is being staged right now
    const len = pieceLength(index, this.info);
    if (offset >= len) return false;
    if (offset + block.length > len) block = block.subarray(0, len - offset); // never into the next piece
    let e = this.#bufs.get(index);
    if (!e) this.#bufs.set(index, e = { bytes: new Uint8Array(len), blocks: new Set() });
    e.bytes.set(block, offset);
    e.blocks.add(Math.floor(offset / 16384));
    if (e.blocks.size < Math.ceil(len / 16384)) return false;
    // a re-sent block of this piece arriving while the stage is pending must not stage (and queue) it twice
    this.#staging.add(index);
    const bytes = e.bytes;
    try {
      await this._serial(async () => {
        if (this.#pending.length >= this.slots) {            // every slot awaits a flush: make room
          this.forcedFlushes++;
          this._deliver(await this._flushLocked());
        }
        if (this.#cpuMax > 0) this.#held.set(index, bytes);   // staged (or hashed on the CPU) by its flush
        else check(this.#l, this.#ctx, await this.#l.symbols.tv_stage(this.#ctx, BigInt(index * this.info.pieceLength), ptr(bytes), BigInt(len)));
        if (this.#pending.length === 0) {
          this.#oldest = performance.now();
          // the age bound also holds when no further block arrives
          if (this.#flushAgeMs !== null) this._armTimer(this.#flushAgeMs);
        }
        this.#pending.push(index);
        this.#pendingSet.add(index);
      });
    } finally {
      this.#staging.delete(index);
    }
    this.#bufs.delete(index);
    await this._autoFlush();                                  // the count bound
    return true;
  }

  private _armTimer(delayMs: number): void {
    clearTimeout(this.#timer);
    this.#timer = setTimeout(() => {
      if (this.#closed || this.#pending.length === 0) return;
      // timers are millisecond-granular and may fire a little before the oldest piece is flushAgeMs old:
      // then wait out the rest instead of leaving the pending pieces to the next block
      const wait = (this.#flushAgeMs || 0) - (performance.now() - this.#oldest);
      if (wait > 0) {
        this._armTimer(Math.max(1, Math.ceil(wait)));
        return;
      }
      this._autoFlush().catch((e) => {
        this.#timerError = e;
      });
    }, delayMs);
  }

  private _open(): void {
    if (this.#closed) throw new Error("PieceVerifier: closed");
  }

  private _rethrow(): void {
    if (this.#timerError !== null) {
      const e = this.#timerError;
      this.#timerError = null;
      throw e;
    }
  }

  /** Would the policy flush now? */
  due(): boolean {
    if (this.#pending.length === 0) return false;
    if (this.#flushPieces !== null && this.#pending.length >= this.#flushPieces) return true;
    return this.#flushAgeMs !== null && performance.now() - this.#oldest >= this.#flushAgeMs;
  }

  /** Results of an automatic or forced flush: to onVerified, else kept for flush() / poll(). */
  private _deliver(res: [number, boolean][]): void {
    if (this.#onVerified) for (const [i, ok] of res) this.#onVerified(i, ok);
    else this.#results.push(...res);
  }

  private async _autoFlush(): Promise<void> {
    if (!this.due()) return;
    this.autoFlushes++;
    await this._serial(async () => this._deliver(await this._flushLocked()));
  }

  /** One list launch over every pending piece (inside a _serial job); frees their slots. */
  private async _flushLocked(): Promise<[number, boolean][]> {
    if (this.#pending.length === 0) return [];
    clearTimeout(this.#timer);
    const pending = this.#pending;
    this.#pending = [];
    this.#pendingSet.clear();
    if (this.#cpuMax > 0) {
      const held = pending.map((i) => this.#held.get(i)!);
      for (const i of pending) this.#held.delete(i);
      if (pending.length <= this.#cpuMax) {   // a short flush: the reference's WebCrypto SHA-1 on the CPU
        const oks = await Promise.all(pending.map((i, k) => cpuPieceOk(held[k], this.info.pieces[i])));
        const res: [number, boolean][] = pending.map((i, k) => [i, oks[k]]);
        for (const [i, good] of res) if (good) this.bitfield[i >> 3] |= 128 >> (i % 8);
        return res;
      }
      for (let k = 0; k < pending.length; k++) {   // a long one: stage the held pieces, one list launch
        check(this.#l, this.#ctx, await this.#l.symbols.tv_stage(this.#ctx, BigInt(pending[k] * this.info.pieceLength),
                                                                 ptr(held[k]), BigInt(held[k].length)));
      }
    }
    const idx = BigUint64Array.from(pending.map(BigInt));
    const ok = new Uint8Array(idx.length);
    check(this.#l, this.#ctx, await this.#l.symbols.tv_verify_list(this.#ctx, ptr(new Uint8Array(idx.buffer)), BigInt(idx.length), ptr(ok)));
    const out: [number, boolean][] = pending.map((i, k) => [i, ok[k] === 1]);
    for (const [i, good] of out) if (good) this.bitfield[i >> 3] |= 128 >> (i % 8);
    return out;
  }

  /** Verify all completed pieces in one launch; returns [index, ok] (after the results of automatic
   * flushes not yet handed out, including one still running when flush() was called) and sets the have-bits. */
  async flush(): Promise<[number, boolean][]> {
    this._open();
    this._rethrow();
    return await this._serial(async () => {
      const earlier = this.#results;
      this.#results = [];
      return [...earlier, ...await this._flushLocked()];
    });
  }

  /** For a client's event loop: flush if the policy says so, and hand out every result the automatic and
   * forced flushes have not yet returned (none when onVerified is set).  As the Python verifier's poll(). */
  async poll(): Promise<[number, boolean][]> {
    this._open();
    this._rethrow();
    await this._autoFlush();
    return await this._serial(async () => {
      const out = this.#results;
      this.#results = [];
      return out;
    });
  }

  /** Release the device context once every library call already queued -- an automatic flush the age timer
   * started included -- has finished (tv_destroy must not run beside a nonblocking call on the same context).
   * Pending pieces not yet flushed are dropped; the verifier cannot be used afterwards. */
  async close(): Promise<void> {
    if (this.#closed) return;
    this.#closed = true;
    clearTimeout(this.#timer);
    await this.#busy;
    this.#l.symbols.tv_destroy(this.#ctx);
  }
}
