#!/bin/bash
# Round 6: does a compact, reused read destination keep the box's reused-buffer O_DIRECT rate?  The C reader into its
# own buffer then memcpy'd to the 192 MiB spread, or DMA'd to the GPU from two page-locked buffers per reader, beside
# the plain and spread readers and the library's cold verify_files (tools/cold_sweep.py COLD_BOUNCE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r06_bounce}
mkdir -p $out /tmp/cs
COLD_BOUNCE=1 COLD_ROUNDS=${COLD_ROUNDS:-2} timeout -k 10 900 python3 -u tools/cold_sweep.py /tmp/cs single16 files64 \
    > $out/cold_bounce.jsonl 2> $out/cold_bounce.err
rc=$?
cat $out/cold_bounce.jsonl; tail -5 $out/cold_bounce.err
exit $rc
