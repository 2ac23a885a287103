/*
 * torrent_verify.h -- C ABI of the MI355X piece-verification engine (libtorrent_verify.so).
 *
 * The reference (rclarey/torrent, TypeScript for Deno) has no verify function and no FFI:
 * its only per-piece SHA-1 is `crypto.subtle.digest("SHA-1", content)` inside
 * tools/make_torrent.ts:28-31.  This ABI is what a Deno `Deno.dlopen` binding of the new
 * verify path (ts/verify.ts) binds.  Each entry point names the reference
 * interface whose data it consumes or replaces.
 *
 * Conventions
 *   - Only fixed-width integers and plain pointers cross the boundary.
 *   - Every function returns TV_OK (0) or a negative TV_ERR_*; the message is available from
 *     tv_last_error().  (The TS/Python host turns a negative status into a thrown Error, like
 *     piece.ts:21-65; unreadable data is NOT an error: it yields a 0 bit, like Storage.get
 *     returning null, storage.ts:50-65.)
 *   - One tv_ctx drives one GPU (one process or host thread per GPU).  Calls on one ctx are
 *     serialised by an internal mutex; different ctxs are independent.
 *   - The caller owns every host pointer and keeps it valid for the duration of the call.
 *     The library owns its HIP streams, events, pinned staging buffers and device memory.
 *   - Piece indices are GLOBAL torrent piece indices; a ctx holds the shard
 *     [shard_first, shard_first + shard_count) resident in HBM.
 *   - Bitfields are MSB-first, piece i -> byte i>>3, mask 0x80>>(i&7), spare bits 0
 *     (reference torrent.ts:53,60 and :147-149).
 */
#ifndef TORRENT_VERIFY_H
#define TORRENT_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TV_ABI_VERSION 1

#define TV_OK 0
#define TV_ERR_ARG (-1)     /* invalid argument / geometry */
#define TV_ERR_HIP (-2)     /* HIP runtime failure (message has the hipError string) */
#define TV_ERR_STATE (-3)   /* call out of order (e.g. verify before set_layout) */
#define TV_ERR_NOMEM (-4)   /* device or pinned host allocation failed */
#define TV_ERR_IO (-5)      /* tv_stage_file: file missing, unreadable or shorter than the read
                               (the reference's fsStorage.get -> null, storage.ts:163-171) */

typedef struct tv_ctx tv_ctx;

/* ABI version of the loaded library (== TV_ABI_VERSION). */
int tv_abi_version(void);

/* Number of visible HIP devices. */
int tv_device_count(int *count);

/* Host CPUs this process may use, as the library sees them (no HIP call, no context): the cgroup CPU quota
 * (cpu.max, v2; cpu.cfs_quota_us / cfs_period_us, v1) when one is set, else OMP_NUM_THREADS when set (a stated
 * share), else the affinity mask; never more than the affinity mask, at least 1.  Hosts divide it among the shards
 * of a call (TV_OPT_FILE_THREADS per context), as torrent_amd/_cpu.py cpu_share does. */
int tv_cpu_share(uint32_t *cores);

/* Create a context bound to HIP device `device`. */
int tv_create(tv_ctx **out, int device);

/* Release every resource of the context.  NULL is a no-op. */
void tv_destroy(tv_ctx *ctx);

/* Copy the last error message of `ctx` (or of the calling thread when ctx == NULL) into buf.
 * Returns the full message length. */
int tv_last_error(const tv_ctx *ctx, char *buf, size_t n);

/*
 * Geometry of the torrent and of this ctx's shard; allocates the resident payload.
 *
 * Device budget.  The payload (shard_count padded pieces) is allocated whole when it fits
 * TV_OPT_RESIDENT_BUDGET (default: the GPU's free memory at this call less a margin).  A larger shard gets a
 * WINDOWED layout instead, so no shard fails for its size: the allocation holds two buffers (one when the
 * budget holds only one) of W pieces (TV_COUNTER_WINDOW_PIECES), staging fills window k's buffer, and when
 * staging reaches window k + 1 the library hashes window k (kernels into the shard's digest rows) while k + 1
 * stages into the other buffer.  tv_verify / tv_hash end the pass (the open window is hashed, windows never
 * staged get zero digests: bit 0) and compare / return the whole shard.  Rules of a windowed layout: staging
 * (tv_stage, tv_stage_file, tv_fill_synthetic) must ascend window by window -- bytes of a window already
 * hashed this pass are TV_ERR_STATE; tv_stage_files sorts its segments itself; tv_read reads the open window
 * only; tv_verify_list is TV_ERR_STATE; repeated tv_verify / tv_hash reuse the pass's digests, and staging
 * after them starts a new pass.  TV_COUNTER_PAYLOAD_BYTES <= the budget (unless one piece exceeds it).
 * Slot pool.  With TV_OPT_LIST_SLOTS = K the payload holds K piece slots instead of the shard (incremental
 * verify: only the pieces awaiting verification need device memory).  A piece takes a free slot when its
 * first byte is staged and keeps it until tv_verify_list lists it; staging a piece when all K slots are
 * taken is TV_ERR_STATE.  tv_verify / tv_hash / tv_fill_synthetic are TV_ERR_STATE on a slot pool.
 *
 *   total_length : InfoDict.length (metainfo.ts:21,40 / :125 sum of file lengths)
 *   piece_length : InfoDict.pieceLength (metainfo.ts:14)
 *   n_pieces     : InfoDict.pieces.length, the DIGEST count (metainfo.ts:16,111);
 *                  piece i has length piece.ts:16-19 and linear offset i*piece_length
 *                  (torrent.ts:165,186)
 *   shard_first, shard_count : pieces resident on this device; shard_first % 8 == 0 so the
 *                  bitfield slice is whole bytes; any shard_first when shard_count == 0
 * Device and pinned allocations are kept and reused when the new geometry fits them (a run of
 * single-piece layouts allocates once).
 * Replaces: the per-piece Storage.get(i*pieceLength, pieceLength(i)) walk (storage.ts:50-65).
 */
int tv_set_layout(tv_ctx *ctx, uint64_t total_length, uint64_t piece_length, uint64_t n_pieces,
                  uint64_t shard_first, uint64_t shard_count);

/*
 * Expected digests: the raw `info.pieces` byte string (pieces_len bytes; NOT 20*n_pieces when
 * the string is ragged).  Slice i is bytes [20i, 20i+20) as partition(info.pieces, 20)
 * makes it (metainfo.ts:111, _bytes.ts:92-99); a slice shorter than 20 bytes never matches.
 */
int tv_set_digests(tv_ctx *ctx, const uint8_t *pieces, uint64_t pieces_len);

/*
 * Copy `len` payload bytes at LINEAR torrent offset `linear_offset` (the concatenation of the
 * files in info.files order, storage.ts:89-137) into the resident payload.  Bytes outside the
 * shard are ignored.  The copy goes through the library's pinned staging ring and is complete
 * when the call returns.  Pageable memory is copied into the ring by TV_OPT_FILE_THREADS threads; a
 * page-locked source (tv_host_alloc / tv_host_register) is DMA'd directly.  Replaces: fsStorage.get
 * reads feeding Storage.get (storage.ts:150-172).
 */
int tv_stage(tv_ctx *ctx, uint64_t linear_offset, const uint8_t *src, uint64_t len);

/*
 * n tv_stage calls in one: buffer k (srcs[k], lens[k] bytes) holds LINEAR bytes [linear_offsets[k],
 * linear_offsets[k] + lens[k]).  The same clipping, windows (ascending, as consecutive tv_stage calls) and mark
 * clearing apply, in order k = 0 .. n-1; every copy is complete when the call returns.  For a host that holds a
 * batch of pieces as separate buffers (one Storage.get result per piece, storage.ts:50-65): the library packs
 * the buffers shorter than 16 MiB into its pinned ring slots (many per slot) on its own threads, one DMA per
 * run of adjacent bytes, on both staging lanes when they fill two slots of a whole-shard layout, so the caller
 * does no gather copy.  Replaces: a batch of Storage.get results (storage.ts:50-65), one per piece, as
 * verifyPieces collects them; or a multi-file payload's files (10,000 of them stage at ~51 GB/s).
 */
int tv_stage_many(tv_ctx *ctx, uint64_t n, const uint64_t *linear_offsets, const uint8_t *const *srcs,
                  const uint64_t *lens);

/*
 * Stage `len` bytes of the file at `path` (a NUL-terminated path), starting at byte `file_offset`,
 * as LINEAR torrent bytes [linear_offset, linear_offset + len).  This is one file segment of
 * Storage.get's mapping (storage.ts:89-137: path, offset in the file, length) read the way
 * fsStorage.get reads it (storage.ts:150-172: open, seek, read).  The bytes are read by parallel preads
 * (TV_OPT_FILE_THREADS threads, 1-4 MiB requests) into the library's pinned ring, one 64 MiB slot at a time,
 * and DMA'd from the slot to HBM while the next slot is read (53 GB/s end to end from a warm page cache on
 * an MI355X host whose PCIe H2D copy runs at 57.6; profiles/r05).  A part whose bytes are mostly not in the
 * page cache is read with O_DIRECT (faster than buffered reads at disk rates; a filesystem that refuses it
 * is read buffered).  Bytes outside the shard are skipped.  A missing, unopenable or short file (or a read error
 * part-way) returns TV_ERR_IO, and the library marks the pieces Storage.get would return null for
 * (storage.ts:50-65 reads piece by piece): from the piece holding the first byte the file cannot supply
 * to the segment's end.  The whole pieces before that byte are staged and stay readable.  Marked pieces
 * are reported 0 by tv_verify and tv_verify_list until the next tv_set_layout; the host marks nothing.  Unlike
 * fsStorage.get (which opens with create: true, storage.ts:28-32,158) a missing file is never created.
 * The file is opened as fsStorage.get opens it (read + write, storage.ts:28-32,158): a file this process
 * may not write returns TV_ERR_IO, as Deno.open fails there.  len == 0 reads nothing but still checks the
 * open: TV_ERR_IO when fsStorage.get's open would fail (a directory, a missing parent directory, no
 * permission); a missing file in a writable directory succeeds (fsStorage.get would create it; this call
 * creates nothing).
 */
int tv_stage_file(tv_ctx *ctx, const char *path, uint64_t file_offset, uint64_t linear_offset, uint64_t len);

/*
 * Stage MANY file segments in one call: a shard's whole Storage.get mapping (storage.ts:89-137), each
 * segment read as fsStorage.get reads it (storage.ts:150-172).  Segment k is `lens[k]` bytes of file
 * `paths[k]` from byte `file_offsets[k]`, staged as LINEAR bytes [linear_offsets[k], +lens[k]).
 *   - Segments of >= TV_OPT_FILE_DIRECT_MIN bytes (default 32 MiB) take the tv_stage_file path, cut into
 *     256 MiB units dealt to two staging lanes (a helper thread with its own copy stream and pinned ring,
 *     and the calling thread; the TV_OPT_FILE_THREADS readers shared between them), which DMA side by side.
 *   - Shorter ones are packed into the pinned ring's 64 MiB slots. TV_OPT_FILE_THREADS threads read
 *     them (open, pread, close; default 16), and each run of linear-contiguous segments is one DMA.
 *     A slot's DMA overlaps the reads of the next slot. This is the many-small-files case: a
 *     10,000-file torrent is one call, not 10,000.
 * status_out[k] = TV_OK, or TV_ERR_IO when the file is missing, unreadable, not writable or shorter than
 * the segment.  As for tv_stage_file, the library itself marks the pieces Storage.get would return null
 * for (from the piece holding the first unreadable byte to the segment's end; the whole pieces before it
 * are staged), tv_verify reports them 0 until the next tv_set_layout, and the status is informational: a
 * host that cleared every piece a failed segment touches would lose a short file's readable pieces.
 *   - Zero-length segments belong in the list: Storage.get's walk emits them for a file that ends where a
 *     piece starts and for a zero-length file inside a piece (storage.ts:109-110), and fsStorage.get still
 *     opens them (storage.ts:158).  Such a segment reads nothing; its status is TV_ERR_IO exactly when that
 *     open would fail (tv_stage_file, len == 0), and nothing is created.  Its piece, linear_offsets[k] /
 *     piece_length, is then marked unreadable.
 * The call itself returns TV_OK unless an argument or HIP error occurs; the first I/O failure's message is
 * kept for tv_last_error.  Bytes outside the shard are skipped.
 */
int tv_stage_files(tv_ctx *ctx, uint64_t n, const char *const *paths, const uint64_t *file_offsets,
                   const uint64_t *linear_offsets, const uint64_t *lens, int32_t *status_out);

/*
 * Stage the shard's bytes from the torrent's FILE TABLE in one call: the library makes Storage.get's walk
 * (storage.ts:89-137) itself.  File k holds `lengths[k]` bytes and is found at the k-th of the n NUL-terminated
 * paths packed back to back in `paths` (`paths_bytes` bytes in all): [dir, ...info.files[k].path] joined, or
 * [dir, info.name] for a single-file torrent (n = 1).  Files are in info.files order, so file k starts at the sum
 * of the lengths before it.  Every segment of the walk that meets the shard is staged as tv_stage_files stages
 * it, the zero-length segments fsStorage.get still opens included (storage.ts:109-110,158).  status_out[k] (n
 * entries, one per FILE) = TV_ERR_IO when a segment of file k failed, else TV_OK; as for tv_stage_files the
 * library marks the unreadable pieces itself and the status is informational.  A host thus passes its file table
 * (which it may keep across calls) and does no per-file work per call.  TV_ERR_ARG when `paths` holds fewer than
 * n NUL-terminated paths or the lengths overflow 64-bit offsets.
 */
int tv_stage_file_table(tv_ctx *ctx, uint64_t n, const uint64_t *lengths, const char *paths, uint64_t paths_bytes,
                        int32_t *status_out);

/* The inverse of tv_stage: copy `len` resident bytes at LINEAR offset `linear_offset` to host
 * `dst` (HBM as the piece store serving block requests, torrent.ts:164-167 Storage.get).  Bytes
 * outside the shard are left untouched in dst. */
int tv_read(tv_ctx *ctx, uint64_t linear_offset, uint8_t *dst, uint64_t len);

/* Fill the resident shard with the synthetic payload of `seed` (benchmarks / GPU tests):
 * byte at linear offset o = byte (o & 7) of splitmix64(seed, o >> 3), little-endian. */
int tv_fill_synthetic(tv_ctx *ctx, uint64_t seed);

/*
 * Verify every resident piece of the shard (HBM-resident path).
 *   avail_bits : optional (NULL = all readable) shard-relative MSB-first bitfield, ceil(shard_count/8)
 *                bytes; a clear bit forces 0 (Storage.get -> null: missing / short file).
 *   bitfield_out : ceil(shard_count/8) bytes, shard-relative; bit j = piece shard_first + j.
 * Piece i's bit is 1 iff its bytes are readable AND SHA-1(bytes) == info.pieces[i].
 */
int tv_verify(tv_ctx *ctx, const uint8_t *avail_bits, uint8_t *bitfield_out);

/*
 * Verify a LIST of resident pieces (incremental verify on piece completion, SURVEY 8f row f1: the
 * piece-message handler torrent.ts:183-193 is where a completed piece is checked).  pieces[k] are
 * GLOBAL piece indices inside this ctx's shard (any order, duplicates allowed); ok_out[k] = 1 iff
 * SHA-1 of the resident bytes of piece pieces[k] equals info.pieces[pieces[k]], else 0.  Only pieces
 * whose bytes were staged should be listed.  On a slot pool (TV_OPT_LIST_SLOTS) a listed piece without a
 * slot (never staged) is 0, and every listed piece's slot is free again when the call returns.
 * TV_ERR_STATE on a windowed layout.
 */
int tv_verify_list(tv_ctx *ctx, const uint64_t *pieces, uint64_t n, uint8_t *ok_out);

/*
 * Verify the shard from a HOST buffer (end-to-end resume check): `src` holds the
 * shard's linear bytes [shard_first*piece_length, ...) (src_len bytes; pieces extending past
 * src_len are unreadable).  Data streams host -> pinned ring -> HBM over PCIe with copy/compute
 * overlap; no resident payload is needed (set the layout with TV_OPT_RESIDENT = 0).  Device memory: two chunk
 * buffers within TV_OPT_RESIDENT_BUDGET (default 1 GiB), each a column of a window of >= 2,048 pieces, at most
 * 256 MiB; TV_OPT_STREAM_CHUNK instead gives columns of that width across the whole shard.
 */
int tv_verify_host(tv_ctx *ctx, const uint8_t *src, uint64_t src_len, const uint8_t *avail_bits,
                   uint8_t *bitfield_out);

/*
 * The resume check from the torrent's FILES through the bounded ring (SURVEY 8f row f2 under a small device
 * budget): the stream engine of tv_stream_*, with the library's own readers filling each request's rows straight
 * from the files (the file table as for tv_stage_file_table: n files of lengths[k] bytes, paths NUL-separated in
 * `paths`).  Each row's linear bytes are walked over the files as Storage.get walks them (storage.ts:98-137) and
 * read as fsStorage.get reads them; a piece is 0 exactly when fsStorage.get would return null for it (a byte in a
 * missing, unopenable or short file, a zero-length segment whose open fails, bytes past the files' end) or its
 * SHA-1 differs.  The layout is set with TV_OPT_RESIDENT = 0; device memory: two chunk buffers within
 * TV_OPT_RESIDENT_BUDGET (default 1 GiB), each a column -- a byte range of every piece of a window of >= 2,048 pieces,
 * as wide as the budget allows -- so each row is one long read and every window's SHA-1s advance with each column;
 * a shard far larger than the budget verifies at the staging rate (an explicit TV_OPT_STREAM_CHUNK instead gives
 * columns of that width across the whole shard).  Host memory: the 192 MiB ring.  status_out[k]
 * (n entries) = TV_ERR_IO when a read or open of file k failed.  Nothing is created.
 */
int tv_stream_file_table(tv_ctx *ctx, uint64_t n, const uint64_t *lengths, const char *paths, uint64_t paths_bytes,
                         const uint8_t *avail_bits, uint8_t *bitfield_out, int32_t *status_out);

/* Creation mode (make_torrent.ts:28-31, :147-173): 20-byte SHA-1 of every resident piece of the
 * shard, written to digests_out (20*shard_count bytes), in piece order. */
int tv_hash(tv_ctx *ctx, uint8_t *digests_out);

/*
 * Streamed verify through a BOUNDED pinned ring (end-to-end resume check, SURVEY 8d cfg5: the
 * resume flow Client.add -> Storage -> bitfield -> sendBitfield, client.ts:53-67, torrent.ts:56-60,101).
 * No resident payload and no whole-shard host buffer are needed: the library hands out requests in the
 * order its kernels consume them, the caller (a Storage.get reader, a file reader, a generator) fills
 * each request's pinned staging slot, and the library DMAs it to HBM over PCIe while the kernels hash the
 * previous column.  Host memory in flight is the ring (TV_STREAM_RING_SLOTS x TV_STREAM_SLOT_BYTES).
 *
 *   tv_stream_begin(ctx, avail)          avail: optional shard-relative MSB-first bits (NULL = all)
 *   loop: tv_stream_next(ctx, &req)      req.rows == 0 -> every byte has been requested
 *         fill req.slot (row q at req.slot + q*req.width) and tv_stream_commit(ctx, &req),
 *         or tv_stream_commit_from(ctx, &req, src, src_pitch) to copy the rows from caller memory
 *   tv_stream_end(ctx, bitfield_out)     ceil(shard_count/8) bytes, as tv_verify
 *
 * A request covers `rows` consecutive pieces starting at GLOBAL piece `piece`, and bytes
 * [offset, offset + width) of each (piece-relative; every request of one column has the same offset; with
 * TV_OPT_STREAM_ROWS the offset is 0 and the width the piece length).
 * Row q holds the LINEAR bytes [(piece+q)*piece_length + offset, ...) of length
 * row_bytes(q) = min(width, piece_len(piece+q) - offset), which is `width` for every row except
 * the short last piece's (0 past its end; piece.ts:16-19).  One request is outstanding at a time.  A piece whose bytes cannot be read
 * (Storage.get -> null, storage.ts:50-65) is reported with tv_stream_unreadable and gets bit 0.
 * Calls that use the resident payload fail with TV_ERR_STATE while a stream is active;
 * tv_set_layout / tv_set_digests / tv_stream_abort end it.  Replaces: the per-piece
 * Storage.get + digest loop (storage.ts:50-65, make_torrent.ts:28-31) of a resume check.
 */
#define TV_STREAM_RING_SLOTS 3
#define TV_STREAM_SLOT_BYTES (64ull << 20)
typedef struct tv_stream_req {
    uint64_t piece;   /* GLOBAL index of row 0's piece */
    uint64_t rows;    /* pieces in this request; 0 = the stream is complete */
    uint64_t offset;  /* byte offset inside each piece (the column) */
    uint64_t width;   /* row pitch in `slot`; row q holds tv_row_bytes(q) <= width valid bytes */
    uint8_t *slot;    /* library-owned page-locked staging memory, rows * width bytes */
    uint64_t seq;     /* request number (tv_stream_commit checks it) */
} tv_stream_req;
int tv_stream_begin(tv_ctx *ctx, const uint8_t *avail_bits);
int tv_stream_next(tv_ctx *ctx, tv_stream_req *req);
int tv_stream_commit(tv_ctx *ctx, const tv_stream_req *req);
/* Rows from caller memory: row q at src + q*src_pitch (row_bytes(q) bytes).  A page-locked src
 * (tv_host_alloc / tv_host_register) is DMA'd directly and must stay unmodified until tv_stream_end /
 * tv_stream_abort returns; pageable memory is copied into the request's slot before the call returns. */
int tv_stream_commit_from(tv_ctx *ctx, const tv_stream_req *req, const uint8_t *src, uint64_t src_pitch);
/* Piece `piece` (GLOBAL, inside the shard) is unreadable: its bit will be 0. */
int tv_stream_unreadable(tv_ctx *ctx, uint64_t piece);
int tv_stream_end(tv_ctx *ctx, uint8_t *bitfield_out);
/* Drop an active stream (a reader failed part-way); the ctx is usable again.  No-op when idle. */
int tv_stream_abort(tv_ctx *ctx);
/* Benchmarks / tests: fill the outstanding request's slot with the synthetic payload of `seed` (the
 * bytes tv_fill_synthetic writes), generated on the host by TV_OPT_FILE_THREADS threads. */
int tv_stream_fill_synthetic(tv_ctx *ctx, const tv_stream_req *req, uint64_t seed);

/* Page-locked host memory for tv_verify_host / tv_stage sources.  A pinned source is read by
 * DMA directly (no staging memcpy); pageable memory goes through the library's pinned ring.
 * tv_host_register pins an existing range (e.g. a caller's buffer), tv_host_unregister undoes it. */
int tv_host_alloc(uint64_t bytes, void **out);
int tv_host_free(void *ptr);
int tv_host_register(void *ptr, uint64_t bytes);
int tv_host_unregister(void *ptr);

/* Options (tv_set_option keys): what a host integrating the library sets.  (Measurement and test knobs -- kernel
 * forcing, stride padding, file-staging A/B modes, NUMA binding, probes, fault injection -- are keys of the
 * library's internal header torrent_amd/csrc/tv_options_internal.h, which only the tests and tools use.) */
#define TV_OPT_STREAM_CHUNK 3 /* tv_verify_host / tv_stream_*: bytes of each piece per streamed column across the
                                 whole shard (0, default: tv_stream_*: the widest power of two <= L whose column over
                                 the shard is <= 512 MiB; tv_verify_host / tv_stream_file_table: windows x columns
                                 within TV_OPT_RESIDENT_BUDGET, or 1 GiB) */
#define TV_OPT_FILE_DIRECT_MIN 7 /* tv_stage_files: segment length that takes the long-segment path (default 32 MiB) */
#define TV_OPT_FILE_THREADS 8    /* host threads of the context (default 16): tv_stage_file(s)' readers (shared by the
                                    two staging lanes), and the copies of pageable tv_stage sources into the pinned
                                    ring.  A host running several contexts in one process divides its CPU share
                                    among them (verify.py / verify.ts do) */
#define TV_OPT_RESIDENT 10       /* 1 (default): tv_set_layout allocates the resident payload; 0: it does not (a
                                    streamed-only ctx, tv_stream_*; the resident calls then fail with TV_ERR_STATE).
                                    Takes effect at the next tv_set_layout */
#define TV_OPT_TWIN_FILL 13      /* twin kernel with fewer workgroups than 2 per CU (resident calls, cfg4's shards at
                                    N = 4 / 8): 1 (default, auto) = add light companion workgroups up to 2 per CU
                                    that run the same instruction stream on one piece of their main workgroup on
                                    the otherwise idle SIMDs and discard the result (a CU running one twin
                                    workgroup is ~4.5 % slower per block than one running two; +2.2-3.2 %, 0.2-0.4 %
                                    more HBM reads) -- unless other processes hold >= 1 GiB of this GPU's memory
                                    (the kernel driver's per-process accounting): on a GPU shared with other work
                                    the companions would take CUs it may be using; 0 = the real grid only, always.
                                    Bitfields are the same either way.  tv_verify_list adds them only to a list of
                                    >= 32 x CUs pieces */
#define TV_OPT_RESIDENT_BUDGET 16 /* bytes of device memory the resident payload may take (0, default: the GPU's free
                                     memory at tv_set_layout less 4 GiB and 64 B per piece).  A shard larger than it
                                     gets a windowed layout (tv_set_layout).  Takes effect at the next tv_set_layout */
#define TV_OPT_LIST_SLOTS 17      /* K > 0: tv_set_layout allocates a pool of K piece slots instead of the shard (see
                                     tv_set_layout; incremental verify, tv_verify_list).  0 (default) = off.  Takes
                                     effect at the next tv_set_layout */
#define TV_OPT_OPEN_RW 18         /* how tv_stage_file(s) open files: 1 (default) = read + write, as fsStorage.get
                                     opens every segment (storage.ts:28-32,158; an unwritable file reads as null);
                                     0 = read-only, as make_torrent.ts:78 opens its sources (creation mode from files
                                     the process may not write).  Zero-length segments' open check follows it */
#define TV_OPT_STREAM_ROWS 19     /* tv_stream_* request rows: 0 (default) = columns of TV_OPT_STREAM_CHUNK bytes of
                                     every shard piece (one launch per column over the whole shard); 1 = whole
                                     pieces (when a piece fits one ring slot), in windows of up to 4 GiB of pieces
                                     per chunk buffer (a multiple of 64 pieces; TV_OPT_RESIDENT_BUDGET / 2 if set
                                     and smaller), one launch per window: one Storage.get per piece for a reader
                                     that opens a file per call (fsStorage.get, storage.ts:149-172).  Set it
                                     before tv_stream_begin (TV_ERR_STATE during a stream) */
#define TV_OPT_CLOCK_PROBE 20     /* 1: verify / hash launches (resident, windows, stream units) record the shader clock
                                     they ran at (workgroup 0 reads the shader and 100 MHz real-time counters at its
                                     start and end; TV_COUNTER_LAST_CLOCK_KHZ).  0 (default) = off */
int tv_set_option(tv_ctx *ctx, int key, int64_t value);
int tv_get_option(tv_ctx *ctx, int key, int64_t *value);

/* Timing of the last tv_verify / tv_hash / tv_verify_host call, from HIP events recorded on the
 * library's compute stream: kernel_ms = the verify kernel(s) only; total_ms = whole call. */
int tv_last_timing(tv_ctx *ctx, double *kernel_ms, double *total_ms);

/* Kernel chosen for the last call (1 lane, 2 split, 4 twin) and launches it used. */
int tv_last_kernel(tv_ctx *ctx, int *kernel, int *launches);

/* Resource counters of a ctx (tv_get_counter keys): how often tv_set_layout and the calls after it had to
 * allocate device memory, and what the ctx holds now.  A run of small layouts on a ctx (verify_piece, list
 * flushes) must not reallocate, and a small call must not evict a bulk call's payload; these make both
 * observable.  No reference counterpart (the reference holds no device memory). */
#define TV_COUNTER_PAYLOAD_ALLOCS 1 /* resident payload allocations since tv_create */
#define TV_COUNTER_DEVICE_ALLOCS 2  /* device allocations of every kind since tv_create */
#define TV_COUNTER_PAYLOAD_BYTES 3  /* bytes of the resident payload allocation held now (0: none) */
#define TV_COUNTER_DEVICE_BYTES 4   /* bytes of device memory held now */
#define TV_COUNTER_LAST_WORKGROUPS 5 /* workgroups of the last verify / hash / list launch (companion
                                        workgroups of TV_OPT_TWIN_FILL included) */
#define TV_COUNTER_NUMA_NODE 6       /* the GPU's NUMA node (sysfs numa_node of its PCI function); UINT64_MAX if
                                        unknown */
#define TV_COUNTER_RING_NODE 7       /* the NUMA node holding the first pinned ring slot's first page; UINT64_MAX
                                        if the ring is not allocated yet or the node is unknown */
#define TV_COUNTER_WINDOW_PIECES 8   /* pieces per window of a windowed layout (0: the shard is resident whole) */
#define TV_COUNTER_WINDOWS 9         /* windows hashed by the current (or last) pass of a windowed layout */
#define TV_COUNTER_BUDGET 10         /* the device budget the last tv_set_layout applied, bytes (0: no resident payload
                                        or a slot pool) */
#define TV_COUNTER_SLOTS_USED 11     /* slots of a slot pool holding a staged piece not yet listed */
#define TV_COUNTER_LAST_CLOCK_KHZ 12 /* TV_OPT_CLOCK_PROBE: the shader clock of the last probed launch's workgroup 0, kHz
                                        (shader-counter ticks / 100 MHz real-time ticks over its life); 0 = none.
                                        Waits for the ctx's queued kernels */
int tv_get_counter(tv_ctx *ctx, int key, uint64_t *value);

/* Block until all work queued by the ctx is complete. */
int tv_synchronize(tv_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* TORRENT_VERIFY_H */
