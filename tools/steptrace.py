"""One training step of a rocprofv3 --kernel-trace run, launch by launch.

    python tools/steptrace.py <run_kernel_trace.csv> [--step -2] [--grep NAME]

Steps are delimited by the Adam launch (adam_kernel / adam_dev_kernel, the last kernel of a
step); --step picks one of them (default: the second-to-last complete one).  Prints every
launch of that step in order (duration, grid, name) and the per-family totals, so a
per-layer figure (which BN pass of which layer) can be read off the order of the model.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)I", n)
    if m:
        n = m.group(1)
    return n.split("(")[0][:90]


def load(path):
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("Name")
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
        wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or ""
        out.append((t0, t1, name, grid, wg))
    out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--grep", default=None)
    ap.add_argument("--quiet", action="store_true", help="families only")
    a = ap.parse_args()
    ks = load(a.trace)
    ends = [i for i, k in enumerate(ks) if "adam_kernel" in k[2] or "adam_dev_kernel" in k[2]]
    if len(ends) < 2:
        raise SystemExit("fewer than two Adam launches in the trace")
    j = ends[a.step]
    i = ends[ends.index(j) - 1] + 1
    step = ks[i:j + 1]
    wall = (step[-1][1] - step[0][0]) / 1e3
    busy = sum(k[1] - k[0] for k in step) / 1e3
    print(f"step: {len(step)} launches, wall {wall:.1f} us, kernel time {busy:.1f} us")
    fam = defaultdict(lambda: [0, 0.0])
    for t0, t1, name, grid, wg in step:
        s = short(name)
        d = (t1 - t0) / 1e3
        fam[s][0] += 1
        fam[s][1] += d
        if not a.quiet and (a.grep is None or a.grep in s):
            print(f"{d:9.1f} us  grid {grid:>9} x {wg:>4}  {s}")
    print("\nper family (us/step, launches):")
    for s, (n, d) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"{d:9.1f} {n:4d}  {s}")


if __name__ == "__main__":
    main()
