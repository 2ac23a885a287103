set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03_ab
KERNEL=1 GIB=200 REPS=5 timeout -k 10 500 python3 tools/variant_bench.py 51200 r02 r03 > gpurun_out/r03_ab/cfg4_lane.jsonl 2>&1 &&
KERNEL=4 GIB=16 REPS=7 timeout -k 10 300 python3 tools/variant_bench.py 16384 r02 r03 > gpurun_out/r03_ab/cfg2_twin.jsonl 2>&1
rc=$?
cat gpurun_out/r03_ab/*.jsonl
exit $rc
