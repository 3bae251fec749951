"""Print per-kernel SQ counter means (per dispatch) from rocprofv3 --pmc pass directories."""
import collections
import csv
import glob
import re
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            m = re.search(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"])
            k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    if "wgrad_reduce" in k or "weight_prep" in k:
        continue
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c in sorted(mean):
        print(f"   {c:28s} {mean[c]:16.0f}")
    w = mean.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_VALU"):
            if c in mean:
                print(f"   {c:28s} {mean[c] / w:8.3f} of SQ_WAVE_CYCLES")
    g = mean.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
        print(f"   mfma busy frac {mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
    if "SQ_LDS_IDX_ACTIVE" in mean and "SQ_LDS_BANK_CONFLICT" in mean:
        print(f"   lds conflict frac {mean['SQ_LDS_BANK_CONFLICT'] / max(1, mean['SQ_LDS_IDX_ACTIVE']):.3f}")
