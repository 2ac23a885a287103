#!/bin/bash
# Round-3 late check on the final build: the whole -m gpu suite, smoke(), cfg3 end to end (the library now
# marks a failed file segment's pieces itself), the default bench line and its rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r03_check3}
mkdir -p $out /tmp/cfg3files
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python tools/cfg3_bench.py /tmp/cfg3files > $out/cfg3_bench.log 2>&1 && echo CFG3_OK &&
timeout -k 10 500 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/bench_prof.json 2> $out/bench_prof.err && echo PROF_OK
rc=$?
tail -3 $out/pytest_gpu.log; cat $out/cfg3_bench.log; head -c 900 $out/bench_n1.json
exit $rc
