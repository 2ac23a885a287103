#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench_valu 2>/dev/null &&
timeout -k 10 200 /tmp/ubench_valu > gpurun_out/ubench_valu.log 2>&1 && echo UBENCH_OK &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python tools/quick_bench.py > gpurun_out/quick_bench.log 2>&1 && echo BENCH_OK
rc=$?
cat gpurun_out/quick_bench.log; tail -2 gpurun_out/pytest_gpu.log
exit $rc
