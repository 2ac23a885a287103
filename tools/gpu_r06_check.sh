#!/bin/bash
# Round 6 check: the windowed and cold-read GPU tests, then tools/window_bench.py (window buffers x hash streams
# at small budgets) and tools/cold_sweep.py COLD_LIBBOUNCE (the library's bounce path against its ring path and
# the C reader), each step under its own time limit, stopping at the first failure.  Knobs: CHECK_TESTS, WB_BUDGETS,
# WB_VARIANTS, WB_FILES (verify_files legs), WB_COLD (cold verify_files legs; its value: --cold-variants), SKIP_COLD (no cold sweep).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r06_check}
mkdir -p $out /tmp/cs
timeout -k 10 500 python -u -m pytest ${CHECK_TESTS:-tests/test_gpu_windows.py tests/test_gpu_cold.py} -x -v \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 && echo TESTS_OK &&
mkdir -p /tmp/wf && timeout -k 10 500 python3 -u tools/window_bench.py --budgets ${WB_BUDGETS:-0.5,1,2} --reps 2 \
    --variants ${WB_VARIANTS:-2:1,2:0,3:0,4:0,4:1,4:2,6:0,8:0,8:4} ${WB_FILES:+--files /tmp/wf} ${WB_COLD:+--cold --cold-variants ${WB_COLD}} \
    > $out/window_bench.jsonl 2> $out/window_bench.err && echo WINDOWS_OK && rm -rf /tmp/wf &&
{ [ -n "$SKIP_COLD" ] || { COLD_LIBBOUNCE=1 COLD_ROUNDS=${COLD_ROUNDS:-2} timeout -k 10 700 python3 -u tools/cold_sweep.py \
    /tmp/cs single16 files64 > $out/cold_libbounce.jsonl 2> $out/cold_libbounce.err && echo COLD_OK; }; }
rc=$?
rm -rf /tmp/wf /tmp/cs
tail -3 $out/pytest.log; tail -3 $out/window_bench.err 2>/dev/null; tail -3 $out/cold_libbounce.err 2>/dev/null
exit $rc
