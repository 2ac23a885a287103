#!/bin/bash
# Build tools/mix_probe (links the library's kernel object; run the library build first).
# Optional: NAME=<binary name> and extra hipcc flags for a kernel variant, e.g.
#   NAME=mix_probe_nofence tools/build_mix_probe.sh -DTV_QUEUE_FENCES=0
set -e
cd "$(dirname "$0")/.."
NAME=${NAME:-mix_probe}
KOBJ=torrent_amd/csrc/tv_kernels.hip.o
if [ $# -gt 0 ]; then
    KOBJ=/tmp/${NAME}_kernels.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I include "$@" -c torrent_amd/csrc/tv_kernels.hip -o $KOBJ
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include -x hip -c tools/mix_probe.cpp -o /tmp/${NAME}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/${NAME}.o $KOBJ -o tools/$NAME
