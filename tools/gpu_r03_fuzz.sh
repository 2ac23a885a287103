#!/bin/bash
# The seeded random-layout suite (tests/test_gpu_fuzz.py), the TS binding under Node (tests/test_ts_binding.py)
# and the streamed paths (parallel row reads) on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03_fuzz
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py tests/test_ts_binding.py tests/test_gpu_stream.py \
    -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_fuzz/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/r03_fuzz/pytest.log
exit $rc
