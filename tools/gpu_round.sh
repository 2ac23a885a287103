#!/bin/bash
# one GPU session: smoke, parity tests, quick bench.  Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python tools/quick_bench.py > gpurun_out/quick_bench.log 2>&1 && echo BENCH_OK
rc=$?
tail -5 gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/quick_bench.log 2>/dev/null
exit $rc
