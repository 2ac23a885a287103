#!/bin/bash
# Round-3 profiles:
#  * the split kernel at cfg4's N = 2 per-GPU shard (25,600 x 4 MiB): timing, rocprofv3 kernel trace + stats,
#    PMC passes (cycles per block, waits, LDS bank conflicts, LDS / VALU instruction counts);
#  * companion workgroups: HBM reads per launch (FETCH_SIZE) at 6,400 and 12,800 pieces (cfg4 at N = 8 / 4),
#    companions on (TV_OPT_TWIN_FILL 1) and off (0), with their times.
# Each step has its own limit; the first failure ends the session.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
out="$R/gpurun_out/r03_prof"
mkdir -p "$out"
SP="tools/shard_probe.py --shards 2 --reps 5"
step() { echo "== $1"; }
step plain && timeout -k 10 300 python3 $SP > $out/split25600_plain.json 2> $out/split25600_plain.err &&
step kt && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 $SP > $out/split25600_kt.json 2> $out/split25600_kt.err &&
i=0 &&
for grp in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  step "pmc $i" && timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $out/pmc_split/p$i -o run -- python3 $SP > $out/pmc_split_p$i.json 2> $out/pmc_split_p$i.err || exit 1
done &&
for sh in 8 4; do
  for fill in 1 0; do
    step "fetch shards=$sh fill=$fill" &&
    timeout -k 10 300 python3 tools/shard_probe.py --shards $sh --twin-fill $fill --reps 5 > $out/twin_s${sh}_f${fill}.json 2> $out/twin_s${sh}_f${fill}.err &&
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_twin_s${sh}_f${fill} -o run -- python3 tools/shard_probe.py --shards $sh --twin-fill $fill --reps 3 > $out/pmc_twin_s${sh}_f${fill}.json 2> $out/pmc_twin_s${sh}_f${fill}.err || exit 1
  done
done
j=0 &&
for grp in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  j=$((j+1))
  step "occ pmc $j" && timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $out/pmc_occ/p$j -o run -- python3 tools/twin_occ_pmc.py > $out/pmc_occ_p$j.log 2> $out/pmc_occ_p$j.err || exit 1
done
rc=$?
cat $out/split25600_plain.json $out/twin_s*_f*.json 2>/dev/null
exit $rc
