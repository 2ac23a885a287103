// tv_options_internal.h -- option keys of libtorrent_verify.so that are NOT part of its public ABI
// (include/torrent_verify.h): measurement and test knobs (A/B builds, probes, fault injection).  The tests and the
// tools set them through tv_set_option with these values; a host integrating the library never needs them.
#pragma once

#define TV_OPT_KERNEL 1      /* 0 = auto, 1 = lane, 2 = split (schedule offload), 4 = twin (split with two lanes per
                                piece); 3 is unused (it was MIX, a work queue measured slower than lane, removed) */
#define TV_OPT_STRIDE_PAD 2  /* bytes of padding between resident pieces (default 256; set before tv_set_layout) */
#define TV_OPT_SPLIT_PAIRS 4 /* split and twin kernels: (rounds, helper) wave pairs per workgroup, 0 = auto, 1, 2;
                                3-5 = SIMD-placement probe shapes (tools/twin_occupancy_probe.py) */
#define TV_OPT_FILE_DIRECT 5 /* tv_stage_file(s) long segments: 0 (default, round 5) = parallel preads into the pinned
                                ring; 1 = windows whose pages are mostly cached (mincore) are mapped, registered
                                (hipHostRegister) and DMA'd from the page cache.  Stamped (tools/f2_stamps.py,
                                profiles/r05): hipHostUnregister + munmap cost 4.9 ms per 256 MiB window, more than
                                its 4.7 ms DMA, so 1 runs at 40-43 GB/s where 0 runs at 53 */
#define TV_OPT_FILE_CHUNK 6  /* long segments: bytes per unit dealt to a lane (and per mapped window with
                                TV_OPT_FILE_DIRECT = 1); default 256 MiB, >= 64 KiB */
#define TV_OPT_FILE_CONCURRENT 9 /* tv_stage_files: 1 (default) = long segments on two staging lanes, 0 = one */
#define TV_OPT_FILE_ODIRECT 22   /* pread path: 1 (default) = chunks mostly not in the page cache are read O_DIRECT;
                                    0 = every read buffered; 2 = tests: every O_DIRECT read fails as a filesystem that
                                    refuses it would (EINVAL), so the file must fall back to buffered reads */
#define TV_OPT_DEBUG_REBOUNCE 11 /* tests: 1 = bounce ring-resident sources through the ring again (the staging
                                    path that once raced); slot leases must keep it exact.  Default 0 */
#define TV_OPT_TWIN_PACK 12      /* twin kernel with fewer workgroups than 2 per CU: 1 = launch it on a stream
                                    CU-masked to ceil(workgroups / 2) CUs, two workgroups on each; 0 (default) =
                                    spread over every CU */
/* TV_OPT_TWIN_FILL (public, 13) also takes 2 = companions on every tv_verify_list launch too (measurement only), and
   3 = companions whatever other processes hold on the GPU (the co-tenant check of 1 skipped) */
#define TV_COUNTER_COTENANT_VRAM 120 /* bytes of this GPU's memory other processes hold (KFD: /sys/class/kfd/kfd/proc/
                                        <pid>/vram_<gpu_id>; 0 when unreadable): >= 1 GiB turns auto companions off */
#define TV_OPT_FILE_BOUNCE 25 /* cold long-segment chunks (O_DIRECT): R > 0 (default 2) = R readers per lane, each
                                 reading 4 MiB parts into one of 2 R reused 4 MiB page-locked buffers and queueing the
                                 part's DMA from it (a compact destination: four reads in flight on two lanes, cold
                                 verify_files 20.7-24.8 against the ring's 15.9-19.8 GB/s in three interleaved sweeps,
                                 profiles/r06/cold_*.jsonl); 0 = parallel preads into the lane's 64 MiB ring slot, one
                                 DMA per slot (rounds 4-5) */
#define TV_OPT_WIN_BUFS 23    /* windowed layouts: window buffers, 0 (default) = tv_plan.h kWinBufsDefault (3), else 1..8
                                 (set before tv_set_layout) */
#define TV_OPT_WIN_STREAMS 24 /* windowed layouts: hash streams, the compute stream included, 0 (default) = buffers - 1
                                 (at most 4), else 1..4; 1 = every window hashed on the compute stream, one after the
                                 other (rounds 4-5) */
#define TV_OPT_STREAM_COLD_WINDOW 26 /* tv_stream_file_table on a shard whose files are mostly not in the page cache:
                                        pieces per window, 0 (default) = 512 (rows four times as long as the warm
                                        geometry's 2,048-piece windows), else a multiple of 64 */
#define TV_OPT_STREAM_COLD_READERS 27 /* its reader threads for O_DIRECT rows, 0 (default) = 2 x TV_OPT_FILE_THREADS
                                         (they wait on the disk, not the CPU), else 1..256 */
#define TV_OPT_STREAM_COLD_REQ 28 /* its request size: bytes of rows per ring request, 0 (default) = one ring slot
                                     (64 MiB), else >= 4096 */
#define TV_COUNTER_WINDOW_BUFS 122    /* window buffers of the current windowed layout (0: not windowed) */
#define TV_COUNTER_WINDOW_STREAMS 123 /* its hash streams (1: the compute stream) */
#define TV_COUNTER_KFD_GPU_ID 121    /* the GPU's KFD gpu_id when the co-tenant check can run (reading it probes for this
                                        process's own accounting entry if not yet known); 0: it cannot */
#define TV_OPT_TWIN_FILL_READS 14 /* companion workgroups' loads: 0 (default) = every lane of a companion reads its
                                    main workgroup's first piece (the same instruction stream, 1/32 of the bytes);
                                    1 = the main workgroup's 32 pieces (round 2; 1.14-1.42 x payload of HBM reads) */
#define TV_OPT_NUMA_BIND 15 /* 1 (default) = the library's host threads (file readers, ring copies, the staging
                               helper lane) run on the CPUs of the GPU's NUMA node, and the pinned ring is
                               allocated on that node (slots allocated after the option is set); 0 = unpinned,
                               default placement (the A/B of profiles/r03/f2_numa_ab.jsonl) */
#define TV_OPT_LANE_PAIRS 21 /* lane kernel loads: 0 (default) = auto: a lane's two 64-B blocks of a 128-B line loaded
                                back to back when the launch has >= 256 x CUs pieces (>= 1 wave per SIMD; HBM reads
                                1.0004 instead of 1.023 x payload at 262,144 x 64 KiB), else a 3-deep ring of
                                single blocks; 1 = pairs always; 2 = never */

/* ---- file staging phase clock (tv_files.hip), for the stamped breakdown of tools/f2_stamps.py ---------------------
 * tv_get_counter(TV_COUNTER_FILE_CLOCK + phase): nanoseconds tv_stage_file(s) spent in that phase since the last
 * reset, summed over the two staging lanes (each lane's phases are disjoint in time, so a phase's total over both
 * lanes can exceed the wall time of the call).  tv_set_option(TV_OPT_FILE_CLOCK_RESET, any) zeroes them. */
#define TV_OPT_FILE_CLOCK_RESET 100
#define TV_COUNTER_FILE_CLOCK 100
#define TV_FILE_PHASE_OPEN 0      /* open + fstat of a unit's file (once per file and lane) */
#define TV_FILE_PHASE_MAP 1       /* mmap of a window + the mincore residency check (direct path); the page-cache
                                     residency check of a unit (pread path: 64 sampled pages) */
#define TV_FILE_PHASE_POPULATE 2  /* direct path: MADV_POPULATE_READ of a warm window */
#define TV_FILE_PHASE_REGISTER 3  /* direct path: hipHostRegister of the window's page-cache pages */
#define TV_FILE_PHASE_READ 4      /* pread path: the parallel preads of one ring slot (wall time of the slot) */
#define TV_FILE_PHASE_WAIT 5      /* a ring slot / mapped window waiting for the DMA that last read it */
#define TV_FILE_PHASE_QUEUE 6     /* queueing the slot's / window's DMA (HIP calls) */
#define TV_FILE_PHASE_RELEASE 7   /* direct path: hipHostUnregister + munmap */
#define TV_FILE_PHASE_DRAIN 8     /* the lane's final stream synchronise (its last DMAs) */
#define TV_FILE_PHASE_SMALL 9     /* short segments: the pool's reads of a packed slot */
#define TV_FILE_PHASE_CALL 10     /* wall time of tv_stage_files / tv_stage_file calls */
#define TV_FILE_BYTES_DIRECT 11   /* bytes DMA'd from registered page-cache pages */
#define TV_FILE_BYTES_READ 12     /* bytes read by preads into the ring (long segments) */
#define TV_FILE_BYTES_ODIRECT 13  /* of which read with O_DIRECT (cold chunks, TV_OPT_FILE_ODIRECT) */
#define TV_FILE_ODIRECT_FALLBACKS 14  /* O_DIRECT reads that failed and were read again buffered (that file then reads
                                         buffered on that lane) */
#define TV_FILE_ODIRECT_ERRNO 15  /* the errno of the first of them since the reset (0: none) */
#define TV_FILE_CLOCK_N 16
