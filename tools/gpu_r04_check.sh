#!/bin/bash
# Round-4 check: the new windowed / slot / open-mode tests first (verbose), then the whole -m gpu suite and
# smoke().  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_check}
mkdir -p $out
timeout -k 10 600 python -u -m pytest ${NEW_TESTS:-tests/test_gpu_windows.py tests/test_gpu_slots.py tests/test_gpu_open_modes.py} \
    -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_new.log 2>&1 && echo NEW_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo SMOKE_OK
rc=$?
tail -30 $out/pytest_new.log; tail -5 $out/pytest_gpu.log 2>/dev/null
exit $rc
