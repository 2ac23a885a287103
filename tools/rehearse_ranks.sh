#!/bin/bash
# Rehearse the driver's N > 1 bench path on ONE GPU: torchrun with N ranks, every rank on the same card
# (bench.py places rank r on device LOCAL_RANK % visible devices).  Default workload as the driver runs it:
# cfg2 weak-scaled (one 16 GiB shard per rank), the cfg4 leg (N shards of the 200 GiB torrent resident at once)
# and e2e_cfg5.
# Usage: tools/rehearse_ranks.sh OUTDIR N [N ...]      (each N under its own 600 s limit, the driver's)
set -o pipefail
out=${1:?outdir}; shift
mkdir -p "$out"
for n in "$@"; do
    port=$((29500 + n))
    SECONDS=0
    timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
        --master-addr 127.0.0.1 --master-port "$port" bench.py --gpus "$n" --steps 10 --warmup 3 \
        > "$out/bench_n${n}_ranks_one_gpu.json" 2> "$out/bench_n${n}_ranks_one_gpu.stderr.log"
    rc=$?
    echo "{\"n\": $n, \"rc\": $rc, \"wall_s\": $SECONDS}" | tee -a "$out/rehearsal_wall.jsonl"
    [ $rc -eq 0 ] || exit $rc
done
