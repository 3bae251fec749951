"""Summarise rocprofv3 --pmc counter_collection CSVs: mean counter value per dispatch for
each kernel (name shortened), plus derived ratios.

    python profiles/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv [more.csv ...]
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(conv_\w+|act_\w+|\w+_kernel)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(paths):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if k.startswith("void at::") or "at::native" in r["Kernel_Name"]:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, cs in vals.items():
        d = list(dur[k].values())
        print(f"{k}  dispatches={len(d)} avg_dur_us={sum(d) / len(d) / 1e3:.1f}")
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        for c, v in sorted(avg.items()):
            print(f"    {c:28s} {v:16.1f}")
        if "SQ_WAVE_CYCLES" in avg:
            wc = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    print(f"    {c + '/WAVE_CYCLES':28s} {avg[c] / wc:16.3f}")
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            print(f"    {'LDS conflict share':28s} {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:16.3f}")
        if "GRBM_GUI_ACTIVE" in avg and d:
            print(f"    {'eff clock GHz (GUI/8/dur)':28s} {avg['GRBM_GUI_ACTIVE'] / 8 / (sum(d) / len(d)):16.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
            # busy cycles summed over SIMDs; per-SIMD-cycle utilisation ~ busy / (GUI_ACTIVE/8 * 1024 SIMDs)
            print(f"    {'MFMA busy / (GUI/8*1024)':28s} "
                  f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):16.3f}")
        if "FETCH_SIZE" in avg and d:
            print(f"    {'FETCH GB/s (x2 gfx950)':28s} {2 * avg['FETCH_SIZE'] * 1024 / (sum(d) / len(d)):16.1f}")
        if "WRITE_SIZE" in avg and d:
            print(f"    {'WRITE GB/s':28s} {avg['WRITE_SIZE'] * 1024 / (sum(d) / len(d)):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
