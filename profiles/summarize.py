"""Summarise a rocprofv3 --kernel-trace --stats CSV (per-kernel totals, per-step share)."""
import csv
import sys


def main(path, steps=7, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.2f} ms over {steps} steps = {tot / 1e6 / steps:.2f} ms/step")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
              f"calls/step={int(r['Calls']) / steps:6.1f} avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 7)
