#!/bin/bash
# Round-4 final check of the build: the whole -m gpu suite, smoke(), the default bench line, its rocprofv3 kernel
# trace, the split kernel on cfg4's N = 2 shard (tools/shard_probe.py) under rocprofv3, and the TS host's Storage
# paths (tools/ts_storage_bench.py).  Every GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_final}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 400 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 \
    > $out/bench_prof.json 2> $out/bench_prof.err && echo PROF_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_split -o run -- python3 tools/shard_probe.py --shards 2 \
    > $out/split25600_under_rocprof.json 2> $out/split25600.err && echo SPLIT_PROF_OK &&
mkdir -p /tmp/tsb && UV_THREADPOOL_SIZE=16 timeout -k 10 400 python3 -u tools/ts_storage_bench.py /tmp/tsb single16 cfg3 \
    > $out/ts_storage_bench.jsonl 2> $out/ts_storage_bench.err && echo TS_BENCH_OK
rc=$?
tail -3 $out/pytest_gpu.log; head -c 400 $out/bench_n1.json; echo
exit $rc
