"""Twin kernel at 8,192 and 16,384 pieces of 1 MiB (one / two 2-wave workgroups per CU), 3 verifies each, for
a rocprofv3 --pmc pass: are the extra ns per block at one workgroup per CU extra shader cycles, or a lower
clock?  usage: rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 tools/twin_occ_pmc.py
Companion workgroups are off (TV_OPT_TWIN_FILL = env FILL, default 0), so 8,192 pieces really is one
workgroup per CU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torrent_amd import _native as N  # noqa: E402

L = 1 << 20
for P in (8192, 16384):
    ctx = N.Context(0)
    ctx.set_option(N.TV_OPT_KERNEL, 4)
    ctx.set_option(N.TV_OPT_TWIN_FILL, int(os.environ.get("FILL", "0")))
    ctx.set_layout(L * P, L, P)
    ctx.fill_synthetic(2)
    ctx.set_digests(bytes(20 * P))
    for _ in range(4):
        ctx.verify()
        print(P, round(ctx.last_timing()[0], 3), flush=True)
    ctx.close()
