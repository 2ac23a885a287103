#!/bin/bash
# After a split-kernel change: its parity tests (verify, hash, list mode, streamed columns, edge geometries),
# then the cfg2 bench line and a piece-count sweep of the split variants.  Each step under its own limit.
# usage: tools/gpu_split_check.sh <tag> [SWEEP_PS]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=${1:-split}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "split or 2 or stream or edge or list or tail or shards or matches" > $O/tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-saturating --no-cfg4 > $O/cfg2.json 2> $O/cfg2.err && echo CFG2_OK &&
SWEEP_PS=${2:-6400,12800,16384,25600,32768} timeout -k 10 300 python3 tools/sweep_pieces.py $O/sweep.jsonl > $O/sweep.log 2>&1 && echo SWEEP_OK
rc=$?
tail -3 $O/tests.log; cat $O/cfg2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac_of_piece_ceiling'], d['bitfield_exact'])"; tail -8 $O/sweep.log
exit $rc
