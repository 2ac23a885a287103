#!/bin/bash
# Round 5: VALU issue evidence for the resident verify kernels on THIS build -- one PMC pass of SQ counters (8 SQ
# slots) and GRBM_GUI_ACTIVE (GRBM block, independent) over the bench's cfg2 (twin) and suppl (lane) workloads,
# after listing which of those counters the box's rocprofv3 knows.  tools/r05_sq.py turns them into per-block
# figures (VALU instructions per wave-block, VALU-active share of wave time, shader clock).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_sq}
mkdir -p $out
python3 -c "from torrent_amd import _native; print(_native.build_id())" > $out/build_id.txt || exit 1
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
want="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY"
have=""
for c in $want; do grep -qw "$c" $out/counters_list.txt && have="$have $c"; done
echo "SQ counters available:$have" | tee $out/sq_available.txt
[ -n "$have" ] || { echo "no SQ counters listed"; exit 1; }
for W in ${PMC_WORKLOADS:-cfg2 suppl}; do
  mkdir -p $out/sq_$W
  timeout -s KILL 240 rocprofv3 --pmc $have GRBM_GUI_ACTIVE --output-format csv -d $out/sq_$W/p1 -o run -- \
      python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-saturating --no-cfg4 --no-cfg3 \
      --e2e-steps 0 > $out/sq_$W/p1.json 2> $out/sq_$W/p1.err || { echo "SQ pass $W FAILED"; tail -5 $out/sq_$W/p1.err; exit 1; }
  echo "sq $W ok"
done
echo SQ_OK
