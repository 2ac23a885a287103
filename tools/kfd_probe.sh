set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/kfd
{
ls -la /sys/class/kfd/kfd/ 2>&1 | head -20
echo ---proc
ls /sys/class/kfd/kfd/proc 2>&1 | head
echo ---topology
for n in /sys/class/kfd/kfd/topology/nodes/*; do echo $n; cat $n/gpu_id 2>&1; grep -E "location_id|domain|drm_render_minor" $n/properties 2>&1; done
echo ---with a context
timeout -k 10 60 python3 -c "
import os, time
from torrent_amd import _native
c = _native.Context(0)
c.set_layout(1<<20, 1<<16, 16)
pid = os.getpid()
base = '/sys/class/kfd/kfd/proc'
for p in sorted(os.listdir(base)):
    d = os.path.join(base, p)
    try:
        fs = os.listdir(d)
    except OSError as e:
        print(p, 'ERR', e); continue
    print(p, 'me' if int(p)==pid else '', fs[:20])
    for f in fs:
        if f.startswith('vram_'):
            try: print('  ', f, open(os.path.join(d,f)).read().strip())
            except OSError as e: print('  ', f, 'ERR', e)
c.close()
"
} > gpurun_out/kfd/probe.txt 2>&1
cat gpurun_out/kfd/probe.txt | head -80
