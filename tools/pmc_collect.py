"""Per-kernel hardware counters of bench.py from rocprofv3 --pmc passes (one counter group per
pass, as gpurun and the PMC slot limits require), corrected as MI355X_MICROARCH.md prescribes:

* HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  (KiB counters; gfx950 FETCH_SIZE tallies
  half the bytes of a wide coalesced stream);
* MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024): the busy cycles
  summed over all 1024 SIMDs against the active cycles of one XCD (rocprofv3 sums
  GRBM_GUI_ACTIVE over the 8 XCDs) times the SIMD count -- the `MfmaUtil` expression of
  counter_defs.yaml, DVFS-independent;
* effective clock = GRBM_GUI_ACTIVE / 8 / kernel duration (duration from a separate
  --kernel-trace run of the same command);
* executed MFMA FLOP = busy cycles * 1024 FLOP per SIMD-cycle (bf16 16x16x32: 16384 FLOP in
  16 cycles), cross-checked against the algorithmic FLOP of the dominant launch.

    python tools/pmc_collect.py --trace <kernel-trace dir> --pass <dir> [--pass <dir> ...] > profiles/rN_pmc.json
"""
import argparse
import collections
import csv
import glob
import json
import re

# bench family -> (kernel-name pattern, total grid size in work-items) of the 256->256 res conv
# at 64x64, B=32 (bench.py's dominant kernel).  Forward and data gradient run the same kernel
# on the same grid: a step dispatches it 13 times in the forward (Generator.in_conv + 12 res
# convs), then 13 times in the backward, so in dispatch order launch i is a forward launch when
# (i // FWD_PER_STEP) is even.
# The weight gradient runs on the sliding-row conv3_halo_wgrad2 (256 blocks of 512), 15
# dispatches per step: the 13 256->256 ones first (12 res + Generator.in_conv, backward order),
# then AFE.down2's two.
DOMS = {
    # (r5 names: conv3_halo_fwd3<4, 2, 4, 8, 2, false, SCH, MODE 0, false>; r6 dropped the PRO flag)
    "fwd": (re.compile(r"conv3_halo_fwd3<4, 2, 4, 8, 2(, false)?(, \d, 0, false)?>"), 512 * 512),
    "dgrad": (re.compile(r"conv3_halo_fwd3<4, 2, 4, 8, 2(, false)?(, \d, 0, false)?>"), 512 * 512),
    "wgrad": (re.compile(r"conv3_halo_wgrad2<4(, false)?>"), 256 * 512),
}
FWD_PER_STEP = 13
WGRAD_PER_STEP, WGRAD_RES = 15, 13
RES_FLOP = 2.0 * 32 * 64 * 64 * 256 * 256 * 9     # one res-conv launch, B=32 (154.6 GFLOP)
SIMDS = 1024
XCDS = 8


def family(name):
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def dom_of(name, grid, k):
    """Dominant families of a dispatch; k = its index among the dispatches of the same kernel
    and grid (dispatch order) separates the forward from the data-gradient launches."""
    fams = [f for f, (pat, g) in DOMS.items() if pat.search(name) and grid == g]
    if "fwd" in fams and "dgrad" in fams:
        fams = ["fwd" if (k // FWD_PER_STEP) % 2 == 0 else "dgrad"]
    if fams == ["wgrad"] and k % WGRAD_PER_STEP >= WGRAD_RES:
        fams = []
    return fams


def _rows(paths, key):
    """CSV rows sorted by dispatch order, each with its index among same-kernel, same-grid rows"""
    rows = [r for p in paths for r in csv.DictReader(open(p))]
    rows.sort(key=lambda r: int(r.get(key) or 0))
    seen = collections.Counter()
    for r in rows:
        grid = int(r.get("Grid_Size", 0) or r.get("Grid_Size_X", 0) or 0)
        k = (r["Kernel_Name"], grid)
        yield r, grid, seen[k]
        seen[k] += 1


def counters(dirs):
    """(family, counter) -> [values], ('dom:'+fam, counter) -> [values]; each pass directory
    is its own run, so dispatch order is counted per pass and per counter"""
    out = collections.defaultdict(list)
    for d in dirs:
        paths = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        rows = [r for p in paths for r in csv.DictReader(open(p))]
        for c in sorted({r["Counter_Name"] for r in rows}):
            sub = [r for r in rows if r["Counter_Name"] == c]
            sub.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
            seen = collections.Counter()
            for r in sub:
                grid = int(r.get("Grid_Size", 0) or 0)
                v = float(r["Counter_Value"])
                out[(family(r["Kernel_Name"]), c)].append(v)
                for f in dom_of(r["Kernel_Name"], grid, seen[(r["Kernel_Name"], grid)]):
                    out[("dom:" + f, c)].append(v)
                seen[(r["Kernel_Name"], grid)] += 1
    return out


def durations(d):
    out = collections.defaultdict(list)
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    for r, grid, k in _rows(paths, "Start_Timestamp"):
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        out[family(r["Kernel_Name"])].append(ns)
        for f in dom_of(r["Kernel_Name"], grid, k):
            out["dom:" + f].append(ns)
    return out


def mean(v):
    return sum(v) / len(v) if v else None


def summarize(cnt, dur, key):
    f = mean(cnt.get((key, "FETCH_SIZE"), []))
    w = mean(cnt.get((key, "WRITE_SIZE"), []))
    busy = mean(cnt.get((key, "SQ_VALU_MFMA_BUSY_CYCLES"), []))
    gui = mean(cnt.get((key, "GRBM_GUI_ACTIVE"), []))
    ns = mean(dur.get(key, []))
    s = {"dispatches": len(dur.get(key, [])) or len(cnt.get((key, "GRBM_GUI_ACTIVE"), [])),
         "avg_us": ns / 1e3 if ns else None}
    if f is not None and w is not None:
        s["read_bytes"] = 2 * f * 1024
        s["write_bytes"] = w * 1024
        s["hbm_bytes_per_launch"] = s["read_bytes"] + s["write_bytes"]
    if busy is not None and gui:
        s["mfma_busy_cycles"] = busy
        s["active_cycles_per_xcd"] = gui / XCDS
        s["mfma_busy_frac"] = busy / (gui / XCDS * SIMDS)
        s["executed_mfma_flop"] = busy * 1024
        if ns:
            s["eff_clock_ghz"] = gui / XCDS / ns
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--pass", dest="passes", action="append", required=True)
    ap.add_argument("--label", default="bench.py --steps 2 --warmup 1 --cpu-seconds 0")
    a = ap.parse_args()
    cnt = counters(a.passes)
    dur = durations(a.trace)
    out = {"source": f"rocprofv3 --pmc passes {a.passes} and --kernel-trace {a.trace} over {a.label}",
           "corrections": __doc__.split("\n\n")[0], "dominant": {}, "families": {}, "step": {}}
    for fam, (pat, g) in DOMS.items():
        s = summarize(cnt, dur, "dom:" + fam)
        shown = re.sub(r"\(.*\)\?", "", pat.pattern)     # the pattern without its optional groups
        s["kernel"] = f"{shown} grid {g} @64x64 B=32 (res conv {fam})"
        s["algorithmic_flop"] = RES_FLOP
        out["dominant"][fam] = s
    fams = sorted({k for k, _ in cnt if not k.startswith("dom:")} | {k for k in dur if not k.startswith("dom:")})
    tot_busy = tot_gui = tot_ns = 0.0
    for k in fams:
        s = summarize(cnt, dur, k)
        out["families"][k] = s
        b = sum(cnt.get((k, "SQ_VALU_MFMA_BUSY_CYCLES"), []))
        gsum = sum(cnt.get((k, "GRBM_GUI_ACTIVE"), []))
        tot_busy += b
        tot_gui += gsum
        tot_ns += sum(dur.get(k, []))
    if tot_gui:
        # GRBM_GUI_ACTIVE over-counts dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS
        # give-back): the all-kernel figure is biased by the step's ~150 short launches, so it
        # is reported with that caveat and bench.py does not quote it
        out["step"] = {"mfma_busy_frac_all_kernels": tot_busy / (tot_gui / XCDS * SIMDS),
                       "eff_clock_ghz_all_kernels": (tot_gui / XCDS) / tot_ns if tot_ns else None,
                       "caveat": "short-dispatch bias of GRBM_GUI_ACTIVE; read the per-family records"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
