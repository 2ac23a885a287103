#!/bin/bash
# Round 5: HBM traffic of the resident verify kernels on THIS build: PMC passes (one counter
# group per pass) over the bench's cfg2 and suppl workloads; the build id compiled into the library is recorded
# so tools/r05_traffic.py writes it into profiles/traffic_<w>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r05_pmc}
mkdir -p $out
python3 -c "from torrent_amd import _native; print(_native.build_id())" > $out/build_id.txt || exit 1
for W in ${PMC_WORKLOADS:-cfg2 suppl}; do
  i=0
  for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
    i=$((i+1))
    mkdir -p $out/pmc_$W
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/pmc_$W/p$i -o run -- \
        python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-saturating --no-cfg4 --no-cfg3 \
        --e2e-steps 0 > $out/pmc_$W/p$i.json 2> $out/pmc_$W/p$i.err || { echo "PMC $W pass $i FAILED: $grp"; tail -5 $out/pmc_$W/p$i.err; exit 1; }
    echo "pmc $W pass $i ok: $grp"
  done
done
echo PMC_OK
