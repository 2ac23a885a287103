#!/bin/bash
# Round-3 second check: the -m gpu suite on the pinned-loop build, cfg3 end to end (verify_payload and
# verify_files over 10,000 files), then the default bench line.  Each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r03_check2
mkdir -p $out /tmp/cfg3files
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python tools/cfg3_bench.py /tmp/cfg3files > $out/cfg3_bench.log 2>&1 && echo CFG3_OK &&
timeout -k 10 500 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK
rc=$?
tail -3 $out/pytest_gpu.log; cat $out/cfg3_bench.log; head -c 600 $out/bench_n1.json
exit $rc
