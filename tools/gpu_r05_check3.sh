#!/bin/bash
# Round 5 check 3 (O_DIRECT cold reads): the -m gpu suite (packed tv_stage_many, unstaged windows, slot pool on two lanes), the default bench
# under rocprofv3 --kernel-trace (per-dispatch durations of every leg, cfg3's included), the Storage-path bench with
# buffered / O_DIRECT / after-legs cold ceilings, and the TS host's Storage paths (verifyPieces hands its batches
# to the packed tv_stage_many).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_check3}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 \
    > $out/bench_prof.json 2> $out/bench_prof.err && echo PROF_OK &&
d=$(python3 tools/fsutil.py pick /tmp/sp "$HOME/sp" /var/tmp/sp 2> $out/evict_probe.json) &&
timeout -k 10 600 python3 -u tools/storage_paths_bench.py "$d" > $out/storage_paths.jsonl 2> $out/storage_paths.err && echo SP_OK
rc=$?
rm -rf /tmp/sp "$HOME/sp" /var/tmp/sp /tmp/tsb
tail -3 $out/pytest_gpu.log; head -c 300 $out/bench_prof.json; echo
exit $rc
