#!/bin/bash
# Split helper waits (stamps, STAMP=2) and the helper-wait-mid variant against the shipped library at cfg4's N = 2
# shard, alternating; the variant's split parity tests.  usage: bash tools/gpu_r04_stamps2.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r04_stamps2}
mkdir -p "$out"
V=build/variants
TORRENT_VERIFY_LIB=$V/libtv_stamps2.so timeout -k 10 120 python3 -u tools/split_stamps.py >> "$out/stamps2_25600.jsonl" || exit 1
TORRENT_VERIFY_LIB=$V/libtv_hmidst.so timeout -k 10 120 python3 -u tools/split_stamps.py >> "$out/hmid_stamps_25600.jsonl" || exit 1
TORRENT_VERIFY_LIB=$V/libtv_hmid.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu > "$out/hmid_parity.log" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 -u tools/split_stamps.py --reps 5 >> "$out/ab_25600.jsonl" || exit 1
  TORRENT_VERIFY_LIB=$V/libtv_hmid.so timeout -k 10 120 python3 -u tools/split_stamps.py --reps 5 >> "$out/ab_25600.jsonl" || exit 1
done
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/split_stamps.py --pieces 32768 --piece-mib 1 --shards 1 --reps 5 >> "$out/ab_32768.jsonl" || exit 1
  TORRENT_VERIFY_LIB=$V/libtv_hmid.so timeout -k 10 120 python3 -u tools/split_stamps.py --pieces 32768 --piece-mib 1 --shards 1 --reps 5 >> "$out/ab_32768.jsonl" || exit 1
done
echo STAMPS2_OK
