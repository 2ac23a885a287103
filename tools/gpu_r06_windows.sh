#!/bin/bash
# Round 6: windows hashed side by side -- the windowed-layout GPU tests, then tools/window_bench.py over window
# buffers x hash streams at small budgets (cfg2's 16 GiB of 1 MiB pieces from page-locked memory).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r06_windows}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_windows.py -x -v --timeout 120 --timeout-method thread \
    > $out/pytest_windows.log 2>&1 && echo TESTS_OK &&
timeout -k 10 500 python3 -u tools/window_bench.py --budgets ${WB_BUDGETS:-0.5,1,2} --reps 2 \
    --variants ${WB_VARIANTS:-2:1,2:0,3:0,4:0,4:1,4:2,6:0,8:0,8:4} > $out/window_bench.jsonl 2> $out/window_bench.err &&
echo BENCH_OK
rc=$?
tail -5 $out/pytest_windows.log; cat $out/window_bench.jsonl; tail -3 $out/window_bench.err
exit $rc
