"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv files)
with derived metrics: MFMA busy % (SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMD x CUs x
GRBM_GUI_ACTIVE / XCDs)), wave wait fractions, LDS conflicts, L2 hit rate, HBM bytes.

    python scripts/pmc_summary.py gpurun_out/pmc_train [--cus 256] [--filter wgrad,conv3x3_train]
"""
import argparse
import collections
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--cus", type=int, default=256)
ap.add_argument("--filter", default="")
a = ap.parse_args()
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
flt = [x for x in a.filter.split(",") if x]
for k, d in sorted(vals.items()):
    if flt and not any(x in k for x in flt):
        continue
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    out = []
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("GRBM_GUI_ACTIVE"):
        out.append(f"mfma_busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * a.cus * avg['GRBM_GUI_ACTIVE'] / 8) * 100:.1f}%")
    if avg.get("SQ_WAVE_CYCLES"):
        w = avg["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
            if c in avg:
                out.append(f"{c[3:].lower()} {avg[c] / w * 100:.0f}%")
    if "SQ_LDS_BANK_CONFLICT" in avg:
        out.append(f"lds_conflict {avg['SQ_LDS_BANK_CONFLICT'] / 1e6:.2f}M")
    if "SQ_INSTS_LDS" in avg:
        out.append(f"lds_insts {avg['SQ_INSTS_LDS'] / 1e6:.2f}M")
    if "TCC_HIT_sum" in avg:
        h, m = avg["TCC_HIT_sum"], avg.get("TCC_MISS_sum", 0)
        out.append(f"l2_hit {h / max(h + m, 1) * 100:.1f}%")
    if "FETCH_SIZE" in avg:
        out.append(f"fetch {avg['FETCH_SIZE'] / 1e3:.1f}MB(raw)")
    print(f"{k:60s} n={len(next(iter(d.values())))} " + " ".join(out))
