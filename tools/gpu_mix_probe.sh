#!/bin/bash
# GPU box: MIX probe over geometries given as "L P last [pairs lanes seg]" arguments (one quoted string
# each).  Exit status 3 (digest mismatch / watchdog) is a finding, not a fault; anything else stops.
# PROBE=<binary in tools/> (default mix_probe), TAG=<output prefix> (default mp)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PROBE=${PROBE:-mix_probe}
TAG=${TAG:-mp}
i=0
for g in "$@"; do
    i=$((i + 1))
    timeout -k 5 60 tools/$PROBE $g gpurun_out/${TAG}_$i.csv > gpurun_out/${TAG}_$i.txt 2>&1
    rc=$?
    cat gpurun_out/${TAG}_$i.txt
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "probe rc=$rc, stopping"; exit $rc; fi
done
