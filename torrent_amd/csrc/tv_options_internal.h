// tv_options_internal.h -- option keys of libtorrent_verify.so that are NOT part of its public ABI
// (include/torrent_verify.h): measurement and test knobs (A/B builds, probes, fault injection).  The tests and the
// tools set them through tv_set_option with these values; a host integrating the library never needs them.
#pragma once

/* ---- file staging phase clock (tv_files.hip), for the stamped breakdown of tools/f2_stamps.py ---------------------
 * tv_get_counter(TV_COUNTER_FILE_CLOCK + phase): nanoseconds tv_stage_file(s) spent in that phase since the last
 * reset, summed over the two staging lanes (each lane's phases are disjoint in time, so a phase's total over both
 * lanes can exceed the wall time of the call).  tv_set_option(TV_OPT_FILE_CLOCK_RESET, any) zeroes them. */
#define TV_OPT_FILE_CLOCK_RESET 100
#define TV_COUNTER_FILE_CLOCK 100
#define TV_FILE_PHASE_OPEN 0      /* open + fstat of a unit's file (once per file and lane) */
#define TV_FILE_PHASE_MAP 1       /* direct path: mmap of a window + the mincore residency check */
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
#define TV_FILE_CLOCK_N 16
