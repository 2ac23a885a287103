#!/bin/bash
# After a lane-kernel change: its parity tests (lane verify/hash, list kernel, edge geometries, streamed
# columns), then cfg4 on one GPU and the piece-saturated config.  Each step under its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=${1:-lane}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_paths.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "1 or lane or list or edge or stream or full_size or reference" > $O/tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python3 bench.py --workload cfg4 --strong --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/cfg4.json 2> $O/cfg4.err && echo CFG4_OK &&
timeout -k 10 300 python3 bench.py --workload suppl --weak --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-cfg4 > $O/suppl.json 2> $O/suppl.err && echo SUPPL_OK
rc=$?
tail -2 $O/tests.log
for f in cfg4 suppl; do python3 -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', d['value'], r['kernel_ms_avg'], round(r['achieved']/r['valu_peak'],4), d['bitfield_exact'])"; done
exit $rc
