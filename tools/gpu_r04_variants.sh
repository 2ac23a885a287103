#!/bin/bash
# Round 4: lane pair-load variant (correctness, A/B at 262,144 x 64 KiB / 65,536 x 256 KiB / 51,200 x 4 MiB, traffic),
# the split rounds loop without LDS-return waits (timing only) at 25,600 x 4 MiB, and the split kernel's LDS latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_var}
mkdir -p $out
V=build/variants
TORRENT_VERIFY_LIB=$V/libtv_pairs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $out/pairs_tests.log 2>&1 && echo PAIRS_TESTS_OK &&
KERNEL=1 GIB=16 REPS=5 timeout -k 10 300 python3 tools/variant_bench.py 262144,65536 base pairs > $out/ab_lane_16g.jsonl 2>&1 && echo AB16_OK &&
KERNEL=1 GIB=200 REPS=3 timeout -k 10 400 python3 tools/variant_bench.py 51200 base pairs > $out/ab_lane_cfg4.jsonl 2>&1 && echo AB200_OK &&
KERNEL=2 GIB=100 REPS=5 timeout -k 10 400 python3 tools/variant_bench.py 25600 base nowait > $out/ab_split_nowait.jsonl 2>&1 && echo ABNW_OK &&
TORRENT_VERIFY_LIB=$V/libtv_pairs.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_pairs_p262k -o run -- \
    python3 bench.py --workload p262k --steps 2 --warmup 1 --no-cpu-baseline --no-saturating --no-cfg4 --e2e-steps 0 \
    > $out/pmc_pairs_p262k.json 2> $out/pmc_pairs_p262k.err && echo PMC_PAIRS_OK &&
timeout -s KILL 240 rocprofv3 --pmc LdsLatency --output-format csv -d $out/pmc_split_lds -o run -- \
    python3 tools/shard_probe.py --shards 2 --rank 0 --reps 2 --warmup 1 > $out/pmc_split_lds.json 2> $out/pmc_split_lds.err && echo PMC_LDS_OK &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $out/pmc_split_lds2 -o run -- \
    python3 tools/shard_probe.py --shards 2 --rank 0 --reps 2 --warmup 1 > $out/pmc_split_lds2.json 2> $out/pmc_split_lds2.err && echo PMC_LDS2_OK
rc=$?
tail -2 $out/pairs_tests.log; cat $out/ab_lane_16g.jsonl $out/ab_lane_cfg4.jsonl $out/ab_split_nowait.jsonl | cut -c1-400
exit $rc
