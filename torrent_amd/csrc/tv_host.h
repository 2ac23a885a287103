// tv_host.h -- host-only helpers of libtorrent_verify.so (tv_host.cpp, compiled by the host C++ compiler).
#pragma once
#include <stdint.h>

// The synthetic payload on the host (tv_stream_fill_synthetic): byte at linear offset off + j = byte
// ((off + j) & 7), little-endian, of splitmix64(seed, (off + j) >> 3) -- the bytes tv_fill_synthetic's
// device kernel writes.  AVX-512 when the host has it (~6 GB/s per core), scalar otherwise (~3).
void tv_synth_fill_host(uint64_t seed, uint64_t off, uint64_t n, uint8_t* out);

// Copy n bytes into a pinned staging slot.  Large copies (>= 64 KiB, AVX-512 hosts) store non-temporally:
// the slot is read only by the DMA engine, and a plain store would first read every destination line.
// TORRENT_VERIFY_NT_STORES=0 turns the non-temporal paths (this and the generator's) off, for A/B runs.
void tv_copy_host(uint8_t* dst, const uint8_t* src, uint64_t n);
