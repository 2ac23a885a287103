#!/bin/bash
# Companion workgroups, round 3: light companions (every lane reads the copied workgroup's first piece,
# TV_OPT_TWIN_FILL_READS 0) against full ones (1, round 2) and none (TV_OPT_TWIN_FILL 0), at cfg4's per-GPU
# shards for N = 8 / 4 (6,400 / 12,800 x 4 MiB) and 4,096 / 8,192 pieces: kernel time, then HBM reads
# (FETCH_SIZE, doubled per MI355X_MICROARCH.md) and cycles per block (GRBM_GUI_ACTIVE / 8) in PMC passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
out="$R/gpurun_out/r03_comp"
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "companions or agree" --timeout 300 > $out/parity.log 2>&1 || { tail -20 $out/parity.log; exit 1; }
echo PARITY_OK
for rnd in 1 2; do
for sh in 8 4; do
  for mode in "1 0" "1 1" "0 0"; do
    set -- $mode
    timeout -k 10 300 python3 tools/shard_probe.py --shards $sh --twin-fill $1 --fill-reads $2 --reps 5 >> $out/times.jsonl 2>> $out/times.err || exit 1
  done
done
done
echo TIMES_OK
for sh in 8 4; do
  for mode in "1 0" "1 1" "0 0"; do
    set -- $mode
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_s${sh}_f$1_r$2 -o run -- python3 tools/shard_probe.py --shards $sh --twin-fill $1 --fill-reads $2 --reps 3 > $out/pmc_s${sh}_f$1_r$2.json 2> $out/pmc_s${sh}_f$1_r$2.err || exit 1
  done
done
echo PMC_OK
cat $out/times.jsonl
