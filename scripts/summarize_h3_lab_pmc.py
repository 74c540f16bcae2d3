"""SQ counters of the H3 tile lab variants (scripts/gpu_r5n.sh -> gpurun_out/r5n/p1, p2) and of
the product towers (scripts/gpu_r5s.sh -> gpurun_out/r5s/<tag>/p1, p2).

    python scripts/summarize_h3_lab_pmc.py gpurun_out/r5n
    python scripts/summarize_h3_lab_pmc.py gpurun_out/r5s/t_b3456
"""
import collections
import csv
import os
import re
import statistics as S
import sys


def main():
    base = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(os.listdir(base)):
        f = os.path.join(base, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            m = re.search(r"(lab_conv|lab_h3|conv_tower|board16_tower|board_tower)(?:<([\d, ]+)>)?", r["Kernel_Name"])
            if m:
                acc[m.group(1) + ("<" + m.group(2) + ">" if m.group(2) else "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| lab_conv<C, BN, WM, TM, NW, VAR, WPE> | MFMA busy | LDS-array busy | wait_any | wait_inst | "
          "wait_inst_lds | active | LDS instr / MFMA | VALU / MFMA | conflict cycles / LDS cycles |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for k, d in acc.items():
        g = lambda c: S.mean(d[c]) if d.get(c) else float("nan")
        gui = g("GRBM_GUI_ACTIVE") / 8          # per-XCD cycles (rocprofv3 sums the 8 XCDs)
        mf = g("SQ_VALU_MFMA_BUSY_CYCLES") / (256 * 4 * gui)
        lds = g("SQ_LDS_IDX_ACTIVE") / (256 * gui)
        wc = g("SQ_WAVE_CYCLES")
        if d.get("GRBM_GUI_ACTIVE") and d.get("_dur"):
            pass
        print(f"| {k} | {mf:.3f} | {lds:.3f} | {g('SQ_WAIT_ANY') / wc:.3f} | {g('SQ_WAIT_INST_ANY') / wc:.3f} | "
              f"{g('SQ_WAIT_INST_LDS') / wc:.3f} | {g('SQ_ACTIVE_INST_ANY') / wc:.3f} | "
              f"{g('SQ_INSTS_LDS') / g('SQ_INSTS_MFMA'):.2f} | {g('SQ_INSTS_VALU') / g('SQ_INSTS_MFMA'):.2f} | "
              f"{g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f} |")


if __name__ == "__main__":
    main()
