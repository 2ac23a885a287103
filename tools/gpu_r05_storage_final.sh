#!/bin/bash
# Round 5, the file-backed paths on the final build: the stamped f2 breakdown warm and cold, the Storage-path bench
# (cold legs residency-checked; buffered and O_DIRECT ceilings) and the interleaved cold sweep.  Each step under its
# own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_storage_final}
mkdir -p $out
python3 -c "from torrent_amd import _native; print(_native.build_id())" > $out/build_id.txt &&
mkdir -p /tmp/f2 && timeout -k 10 400 python3 -u tools/f2_stamps.py /tmp/f2 > $out/f2_stamps.jsonl 2> $out/f2_stamps.err && echo STAMPS_OK &&
rm -rf /tmp/f2 && d=$(python3 tools/fsutil.py pick /tmp/sp "$HOME/sp" /var/tmp/sp 2> $out/evict_probe.json) &&
timeout -k 10 600 python3 -u tools/storage_paths_bench.py "$d" > $out/storage_paths.jsonl 2> $out/storage_paths.err && echo SP_OK &&
rm -rf "$d" && mkdir -p /tmp/cs && timeout -k 10 300 python3 -u tools/cold_sweep.py /tmp/cs > $out/cold_sweep.jsonl 2> $out/cold_sweep.err && echo COLD_OK
rc=$?
rm -rf /tmp/sp "$HOME/sp" /var/tmp/sp /tmp/f2 /tmp/cs
exit $rc
