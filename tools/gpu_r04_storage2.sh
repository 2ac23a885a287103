#!/bin/bash
# Round-4: the host-path tests after the GIL-free copy / pinned batch changes, then the Storage-path bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_storage2}
mkdir -p $out /tmp/sp
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_fuzz.py tests/test_gpu_paths.py tests/test_gpu_windows.py \
    tests/test_gpu_resources.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 && echo TESTS_OK &&
timeout -k 10 600 python3 -u tools/storage_paths_bench.py /tmp/sp > $out/storage_paths.jsonl 2> $out/storage_paths.err && echo SP_OK
rc=$?
tail -3 $out/pytest.log; cat $out/storage_paths.jsonl; tail -5 $out/storage_paths.err
exit $rc
