#!/bin/bash
# Split-kernel barrier stamps at cfg4's N = 2 shard: the stamped diagnostic library and the
# shipped one alternating, then the stamped one on the cfg2 geometry.  usage: bash tools/gpu_r04_stamps.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r04_stamps}
mkdir -p "$out"
S=build/variants/libtv_stamps.so
for r in 1 2; do
  TORRENT_VERIFY_LIB=$S timeout -k 10 120 python3 -u tools/split_stamps.py >> "$out/stamps_25600.jsonl" || exit 1
  timeout -k 10 120 python3 -u tools/split_stamps.py >> "$out/stamps_25600.jsonl" || exit 1
done
TORRENT_VERIFY_LIB=$S timeout -k 10 120 python3 -u tools/split_stamps.py --pieces 16384 --piece-mib 1 --shards 1 \
  >> "$out/stamps_16384.jsonl" || exit 1
echo STAMPS_OK
