#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only with kernel dispatch rows).
# usage: tools/pmc.sh <workload> <kernel> <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
W=$1; K=$2; TAG=$3
export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc/$TAG"
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
           "TA_BUSY_avr TA_BUSY_max SQ_INST_CYCLES_VMEM" \
           ${PMC_EXTRA:+"$PMC_EXTRA"}; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py --workload $W --kernel $K --steps 2 --warmup 1 --no-cpu-baseline --no-saturating --no-cfg4 --e2e-steps 0 > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "PASS $i FAILED: $grp"; tail -5 "$OUT/p$i.err"; exit 1; }
  echo "pass $i ok: $grp"
done
