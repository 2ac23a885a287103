#!/bin/bash
# Round-4 build check: the whole -m gpu suite, smoke(), the default bench line and its rocprofv3 kernel trace,
# the saturated lane legs' HBM traffic with pair loads (FETCH_SIZE passes), and the flush / CPU crossover table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_round}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 400 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 \
    > $out/bench_prof.json 2> $out/bench_prof.err && echo PROF_OK || exit 1
for W in p262k suppl; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_$W -o run -- \
      python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-saturating --no-cfg4 --e2e-steps 0 \
      > $out/pmc_$W.json 2> $out/pmc_$W.err && echo "PMC_$W OK" || exit 1
done
timeout -k 10 300 python3 tools/cpu_crossover.py > $out/cpu_crossover.json 2> $out/cpu_crossover.err && echo XOVER_OK
rc=$?
tail -3 $out/pytest_gpu.log; head -c 600 $out/bench_n1.json; echo; tail -12 $out/cpu_crossover.json
exit $rc
