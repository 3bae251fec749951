"""Per-step kernel budget from the REPLAYED steps of a rocprofv3 --kernel-trace run only.

    python tools/stepbudget.py <run_kernel_trace.csv> [--top 40] [--json out.json]

A step ends at its Adam launch; graph-replayed steps end with `adam_dev_kernel` (the device
step counter), eager steps (warm-up, the capture's own eager step, the HIP-event timing steps
after the timed region) with `adam_kernel`.  Only steps whose Adam is `adam_dev_kernel` and
whose predecessor step also ended in a replay are averaged, so warm-up and first-step work
never enter the budget.  Prints the kernel time per step, the wall
time per step (first launch start -> Adam end) and the per-kernel / per-family averages.
"""
import argparse
import json
from collections import defaultdict

from steptrace import load, short


def _h3(n, prefix, rest):
    """conv3_halo_fwd3<prefix, [false, ]rest...>: the r5 template had a PRO flag after NSB"""
    return n.startswith(f"conv3_halo_fwd3<{prefix}, false, {rest}") or n.startswith(f"conv3_halo_fwd3<{prefix}, {rest}")


FAMILIES = [
    ("res conv fwd/dgrad", lambda n: _h3(n, "4, 2, 4, 8, 2", "2, 0")),
    ("res+down wgrad", lambda n: n.startswith("conv3_halo_wgrad2")),
    ("wgrad slab reduce", lambda n: "wgrad_reduce" in n or "subpix_split_sum" in n or "subpix_fold" in n
     or "w7_reduce" in n),
    ("BN elementwise", lambda n: n.startswith("act_") or "tensor_stats" in n),
    ("BN record folds", lambda n: n.startswith("fold") or "rec_finalize" in n or "finalize" in n),
    ("7x7 family", lambda n: n.startswith("conv7") or n.startswith("conv_halo_wgrad<7")),
    ("1x1 convs", lambda n: n.startswith("conv_fwd_v2<1") or n.startswith("conv_wgrad_v2<1")
     or n.startswith("conv1x1")),
    ("down1 fwd/dgrad", lambda n: n.startswith("conv3c64_fwd") or n.startswith("conv3_halo_fwd3<1, 8")),
    ("down2 fwd/dgrad", lambda n: _h3(n, "2, 4, 4, 4, 3", "2, 0")),
    ("up family", lambda n: n.startswith("conv3up") or n.startswith("conv3_up_wgrad")
     or _h3(n, "2, 4, 4, 4, 3", "2, 2") or _h3(n, "4, 2, 4, 8, 2", "2, 1")
     or _h3(n, "4, 2, 4, 8, 2", "2, 2")),
]


def family(n):
    for f, p in FAMILIES:
        if p(n):
            return f
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ks = load(a.trace)
    ends = [(i, "adam_dev_kernel" in k[2]) for i, k in enumerate(ks)
            if "adam_kernel" in k[2] or "adam_dev_kernel" in k[2]]
    steps = []
    for j in range(1, len(ends)):
        (i0, dev0), (i1, dev1) = ends[j - 1], ends[j]
        if dev0 and dev1:
            steps.append(ks[i0 + 1:i1 + 1])
    if not steps:
        raise SystemExit("no two consecutive replayed steps in the trace")
    n = len(steps)
    kern = defaultdict(lambda: [0, 0.0])
    fam = defaultdict(lambda: [0, 0.0])
    busy = wall = 0.0
    for st in steps:
        wall += (st[-1][1] - st[0][0]) / 1e3
        for t0, t1, name, _, _ in st:
            s, d = short(name), (t1 - t0) / 1e3
            busy += d
            kern[s][0] += 1
            kern[s][1] += d
            f = family(s)
            fam[f][0] += 1
            fam[f][1] += d
    print(f"{n} replayed steps: kernel time {busy / n / 1e3:.3f} ms/step, wall {wall / n / 1e3:.3f} ms/step, "
          f"{sum(v[0] for v in kern.values()) / n:.0f} launches/step")
    print("\nper family (ms/step, launches/step):")
    for f, (c, d) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"{d / n / 1e3:8.3f} {c / n:6.1f}  {f}")
    print(f"\ntop kernels (us/step, launches/step, us/launch):")
    for s, (c, d) in sorted(kern.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{d / n:9.1f} {c / n:6.1f} {d / c:8.1f}  {s}")
    if a.json:
        json.dump({"replayed_steps": n, "kernel_ms_per_step": busy / n / 1e3, "wall_ms_per_step": wall / n / 1e3,
                   "families_ms": {f: d / n / 1e3 for f, (c, d) in fam.items()},
                   "kernels_us": {s: [c / n, d / n] for s, (c, d) in kern.items()}}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
