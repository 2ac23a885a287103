"""Kernel statistics from a rocprofv3 results database (`rocprofv3 --kernel-trace --stats -d DIR -o run`
writes DIR/run_results.db on this ROCm).

    python tools/rocpd_stats.py DIR/run_results.db OUT.csv [--last KERNEL_SUBSTRING N]

OUT.csv gets the profiler's own per-kernel summary (the `top_kernels` view: name, calls, total, average in
us, percent).  With --last, the average duration of the last N dispatches of the first kernel whose name
contains KERNEL_SUBSTRING is printed too (the bench's timed steps follow its warmup dispatches).
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


if __name__ == "__main__":
    main(sys.argv[1:])
