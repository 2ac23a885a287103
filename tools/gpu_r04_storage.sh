#!/bin/bash
# Round-4: stream row mode tests, the default bench line (cfg2 must be unchanged by the windowing work), and the
# Storage-path / cold-cache measurements (tools/storage_paths_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_storage}
mkdir -p $out /tmp/sp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_fuzz.py tests/test_ts_binding.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > $out/pytest_stream.log 2>&1 && echo STREAM_OK &&
timeout -k 10 300 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK &&
timeout -k 10 600 python3 -u tools/storage_paths_bench.py /tmp/sp > $out/storage_paths.jsonl 2> $out/storage_paths.err && echo SP_OK
rc=$?
tail -3 $out/pytest_stream.log; head -c 700 $out/bench_n1.json; echo; cat $out/storage_paths.jsonl; tail -5 $out/storage_paths.err
exit $rc
