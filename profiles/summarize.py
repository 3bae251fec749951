"""Summarise a rocprofv3 --kernel-trace --stats run (per-kernel totals, per-step share).

    python profiles/summarize.py <kernel_stats.csv | results.db> [steps]

Accepts either the `*_kernel_stats.csv` written with `--output-format csv` or the rocpd
SQLite database rocprofv3 writes by default.
"""
import csv
import sqlite3
import sys


def rows_from(path):
    """-> [(name, calls, total_ns, avg_ns)]"""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(r[0], r[1], float(r[2]), float(r[3])) for r in c.execute(
            "select name, count(*), sum(end-start), avg(end-start) from kernels group by name")]
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])))
    return out


def main(path, steps=7, top=40):
    rows = rows_from(path)
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot / 1e6:.2f} ms over {steps} steps = {tot / 1e6 / steps:.2f} ms/step")
    print(f"{'ms/step':>8} {'share':>7} {'calls/step':>10} {'avg_us':>9}  kernel")
    for name, calls, t, avg in sorted(rows, key=lambda r: -r[2])[:top]:
        print(f"{t / 1e6 / steps:8.3f} {100 * t / tot:6.2f}% {calls / steps:10.1f} {avg / 1e3:9.1f}  {name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 7)
