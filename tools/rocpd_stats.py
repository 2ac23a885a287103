"""Kernel statistics from a rocprofv3 results database (`rocprofv3 --kernel-trace --stats -d DIR -o run`
writes DIR/run_results.db on this ROCm).

    python tools/rocpd_stats.py DIR/run_results.db OUT.csv [--last KERNEL_SUBSTRING N] [--dispatches OUT2.csv]

OUT.csv gets the profiler's own per-kernel summary (the `top_kernels` view: name, calls, total, average in
us, percent).  With --last, the average duration of the last N dispatches of the first kernel whose name
contains KERNEL_SUBSTRING is printed too (the bench's timed steps follow its warmup dispatches).  With
--dispatches, every dispatch of the SHA-1 kernels (tv_*_kernel; not the runtime's copy / fill kernels) goes to
OUT2.csv in start order: kernel, start (ns, profiler clock), duration (ns) -- so a per-dispatch average quoted from
the trace (e.g. the timed steps of one bench leg) is reproducible from the tracked file.
"""
import csv
import sqlite3
import sys


def main(argv):
    db, out = argv[0], argv[1]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "calls", "total_us", "average_us", "percent"])
        w.writerows(rows)
    if "--last" in argv:
        k = argv.index("--last")
        sub, n = argv[k + 1], int(argv[k + 2])
        name = next(r[0] for r in rows if sub in r[0])
        durs = [d for (d,) in c.execute("select duration from kernels where name = ? order by start", (name,))]
        tail = durs[-n:]
        print(f"{name}: last {len(tail)} of {len(durs)} dispatches average {sum(tail) / len(tail) / 1e6:.3f} ms")
    if "--dispatches" in argv:
        out2 = argv[argv.index("--dispatches") + 1]
        with open(out2, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "start_ns", "duration_ns"])
            for name, start, dur in c.execute("select name, start, duration from kernels order by start"):
                if name.startswith("void tv_") or name.startswith("tv_"):
                    w.writerow([name, start, dur])


if __name__ == "__main__":
    main(sys.argv[1:])
