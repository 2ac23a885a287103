import os, sys, time, statistics
sys.path.insert(0, "/root/repo")
sys.argv = ["x", "/tmp/tvsf", "16", "16"]
src = open("/root/repo/tools/stage_file_bench.py").read().split("names = {")[0]
exec(src)
res = {}
for rnd in range(4):
    for mode in (1, 0):
        for chunk in (64 << 20, 256 << 20, 1 << 30):
            ctx.set_option(_native.TV_OPT_FILE_DIRECT, mode)
            ctx.set_option(_native.TV_OPT_FILE_CHUNK, chunk)
            t0 = time.perf_counter()
            for k, path in enumerate(paths):
                assert ctx.stage_file(path, 0, k * per, per)
            el = time.perf_counter() - t0
            res.setdefault((mode, chunk), []).append(total / el / 1e9)
for (mode, chunk), v in sorted(res.items()):
    print(f"direct={mode} chunk={chunk >> 20} MiB: median {statistics.median(v):.2f} GB/s  all {[round(x, 1) for x in v]}", flush=True)
