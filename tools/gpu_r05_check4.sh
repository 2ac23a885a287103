#!/bin/bash
# Round 5 check 4: the -m gpu suite (cold / warm O_DIRECT choice), the stamped f2 breakdown warm and cold, the
# Storage-path bench (cold legs residency-checked; buffered and O_DIRECT ceilings), and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_check4}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
mkdir -p /tmp/f2 && timeout -k 10 400 python3 -u tools/f2_stamps.py /tmp/f2 > $out/f2_stamps.jsonl 2> $out/f2_stamps.err && echo STAMPS_OK &&
rm -rf /tmp/f2 && d=$(python3 tools/fsutil.py pick /tmp/sp "$HOME/sp" /var/tmp/sp 2> $out/evict_probe.json) &&
timeout -k 10 600 python3 -u tools/storage_paths_bench.py "$d" > $out/storage_paths.jsonl 2> $out/storage_paths.err && echo SP_OK &&
timeout -k 10 300 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK
rc=$?
rm -rf /tmp/sp "$HOME/sp" /var/tmp/sp /tmp/f2
tail -3 $out/pytest_gpu.log; head -c 300 $out/bench_n1.json; echo
exit $rc
