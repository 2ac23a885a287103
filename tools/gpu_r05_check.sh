#!/bin/bash
# Round 5 check: the -m gpu suite, smoke, the stamped f2 breakdown (single16 / files64 / cfg3), the default bench
# line (now with the cfg3 leg), and the Storage-path bench warm + cold (cold legs residency-checked, in the first
# directory where the page cache can actually be dropped).  Each GPU step has its own limit; the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_check}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK &&
mkdir -p /tmp/f2 && timeout -k 10 400 python3 -u tools/f2_stamps.py /tmp/f2 > $out/f2_stamps.jsonl 2> $out/f2_stamps.err && echo STAMPS_OK &&
rm -rf /tmp/f2 && d=$(python3 tools/fsutil.py pick /tmp/sp "$HOME/sp" /var/tmp/sp "$GRAFT_REPO_ROOT/gpurun_out/sp" 2> $out/evict_probe.json) &&
echo "storage dir: $d" && timeout -k 10 600 python3 -u tools/storage_paths_bench.py "$d" > $out/storage_paths.jsonl 2> $out/storage_paths.err && echo SP_OK
rc=$?
rm -rf /tmp/sp "$HOME/sp" /var/tmp/sp "$GRAFT_REPO_ROOT/gpurun_out/sp" /tmp/f2
tail -3 $out/pytest_gpu.log; head -c 600 $out/bench_n1.json; echo; cat $out/evict_probe.json; echo
exit $rc
