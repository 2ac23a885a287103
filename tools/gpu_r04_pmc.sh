#!/bin/bash
# Round 4:
#  1. the 4-buffer K+W ring variant (helper three blocks ahead) for correctness (parity tests + cfg2 vs the oracle),
#  2. its A/B against the shipped 3-buffer build: split at 25,600 x 4 MiB (cfg4's N = 2 shard), twin at cfg2,
#  3. PMC passes of the saturated lane kernel (p262k: 262,144 x 64 KiB; suppl: 65,536 x 256 KiB): HBM traffic
#     (FETCH_SIZE; TCC_EA0_RDREQ by size), L2 hits, shader cycles (GRBM_GUI_ACTIVE) -> clock,
#  4. the bench's p262k / suppl lines with the live clock probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_pmc}
mkdir -p $out
V=build/variants
TORRENT_VERIFY_LIB=$V/libtv_bufs4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    "tests/test_gpu_paths.py::test_full_size_cfg2_oracle_ground_truth" -m gpu -x -q --timeout 200 --timeout-method thread \
    > $out/bufs4_tests.log 2>&1 && echo BUFS4_TESTS_OK &&
KERNEL=2 GIB=100 REPS=5 timeout -k 10 400 python3 tools/variant_bench.py 25600 base bufs4 > $out/ab_split_25600.jsonl 2>&1 && echo AB_SPLIT_OK &&
KERNEL=4 GIB=16 REPS=7 timeout -k 10 300 python3 tools/variant_bench.py 16384 base bufs4 > $out/ab_twin_16384.jsonl 2>&1 && echo AB_TWIN_OK || exit 1
for W in p262k suppl; do
  i=0
  for grp in "FETCH_SIZE" \
             "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
             "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/pmc_$W/p$i -o run -- \
        python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-saturating --no-cfg4 --e2e-steps 0 \
        > $out/pmc_$W/p$i.json 2> $out/pmc_$W/p$i.err || { echo "PMC $W pass $i FAILED: $grp"; tail -5 $out/pmc_$W/p$i.err; exit 1; }
    echo "pmc $W pass $i ok: $grp"
  done
  timeout -k 10 300 python3 bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-saturating --no-cfg4 \
      --e2e-steps 0 > $out/bench_$W.json 2> $out/bench_$W.err && echo "BENCH_$W OK" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_p262k -o run -- python3 bench.py --workload p262k --steps 10 \
    --warmup 3 --no-cpu-baseline --no-saturating --no-cfg4 --e2e-steps 0 > $out/bench_p262k_kt.json 2> $out/bench_p262k_kt.err && echo KT_OK
rc=$?
tail -3 $out/bufs4_tests.log; cat $out/ab_split_25600.jsonl $out/ab_twin_16384.jsonl; head -c 1500 $out/bench_p262k.json; echo
exit $rc
