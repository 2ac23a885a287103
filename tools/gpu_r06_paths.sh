#!/bin/bash
# Round 6 host-path measurements of the build: the TS host's Storage paths and verifyFiles phases on cfg3 (the file
# table behind the ABI), small budgets (verify_payload from page-locked memory and verify_files on a 16 GiB file, warm
# and cold, in windows and streamed), and cold verify_files (the default bounce path, the ring path, the C reader)
# interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r06_paths}
mkdir -p $out /tmp/tsb /tmp/tsp /tmp/wf /tmp/cs
UV_THREADPOOL_SIZE=16 timeout -k 10 300 python3 -u tools/ts_storage_bench.py /tmp/tsb single16 cfg3 \
    > $out/ts_storage_bench.jsonl 2> $out/ts_storage_bench.err && echo TS_BENCH_OK && rm -rf /tmp/tsb &&
UV_THREADPOOL_SIZE=16 timeout -k 10 300 python3 -u tools/ts_files_phases.py /tmp/tsp cfg3 8 \
    > $out/ts_files_phases_cfg3.jsonl 2> $out/ts_files_phases.err && echo TS_PHASES_OK && rm -rf /tmp/tsp &&
timeout -k 10 500 python3 -u tools/window_bench.py --budgets 0.25,0.5,1,2 --reps 2 --files /tmp/wf --cold \
    > $out/window_bench.jsonl 2> $out/window_bench.err && echo WINDOWS_OK && rm -rf /tmp/wf &&
COLD_LIBBOUNCE=1 COLD_ROUNDS=${COLD_ROUNDS:-2} timeout -k 10 500 python3 -u tools/cold_sweep.py /tmp/cs single16 files64 \
    > $out/cold_sweep.jsonl 2> $out/cold_sweep.err && echo COLD_OK
rc=$?
rm -rf /tmp/tsb /tmp/tsp /tmp/wf /tmp/cs
tail -n 2 $out/*.err
exit $rc
