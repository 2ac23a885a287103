#!/bin/bash
# Round-3 GPU session: smoke, the whole -m gpu suite, the small-call latency probe (list flushes with and
# without companion workgroups).  Each GPU step has its own time limit; the first failure ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r03_check
mkdir -p $out
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python tools/latency_probe.py 20 > $out/latency.json 2> $out/latency.err && echo LATENCY_OK
rc=$?
tail -3 $out/smoke.log; tail -5 $out/pytest_gpu.log
exit $rc
