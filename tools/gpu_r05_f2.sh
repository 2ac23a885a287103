#!/bin/bash
# Round 5: the -m gpu suite on the split library with the lane-unit file engine, then the stamped verify_files
# breakdown (tools/f2_stamps.py) over file-staging configurations on warm single16 / files64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_f2}
mkdir -p $out /tmp/f2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 600 python3 -u tools/f2_stamps.py /tmp/f2 > $out/f2_stamps.jsonl 2> $out/f2_stamps.err && echo STAMPS_OK
rc=$?
tail -3 $out/pytest_gpu.log; cat $out/f2_stamps.jsonl; tail -5 $out/f2_stamps.err
exit $rc
