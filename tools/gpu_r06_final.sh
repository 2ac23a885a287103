#!/bin/bash
# Round 6 final check of the build: the whole -m gpu suite, smoke(), the default bench line, the PMC traffic passes
# of cfg2 and suppl on THIS build (their build id), the default bench under rocprofv3 --kernel-trace --stats, and the
# driver's torchrun command at N = 2 and 8 rehearsed on the one GPU (the host-path measurements: gpu_r06_paths.sh).
# Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r06_final}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python3 bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK &&
CHECK_OUT=${CHECK_OUT:-r06_final}/pmc bash tools/gpu_r05_pmc.sh > $out/pmc.log 2>&1 && echo PMC_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 \
    > $out/bench_prof.json 2> $out/bench_prof.err && echo PROF_OK &&
bash tools/rehearse_ranks.sh $out/rehearse ${REHEARSE_N:-2 8} && echo REHEARSE_OK
rc=$?
tail -3 $out/pytest_gpu.log; head -c 400 $out/bench_n1.json; echo; tail -3 $out/pmc.log
exit $rc
