"""HBM bytes per launch of the 16x16x32 board tower (board16_tower) from the PMC passes of
scripts/gpu_pmc_board16.sh -> "board16" records in profiles/conv_traffic.json (records of
other kernels / configs are kept; a record with the same config is replaced).  gfx950
corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE x2 (wide coalesced reads are tallied at
half their bytes), KiB -> bytes.  Algorithmic bytes per launch: the layer-by-layer
definition the other tower records use (every conv reads its padded input and weights and
writes its interior output, every second conv reads the residual) -- the board tower keeps
activations in LDS, so its traffic is a fraction of that.

    python scripts/summarize_board16_pmc.py gpurun_out/pmc_b16 r6
"""
import collections
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAGS = {"b512": (6, 128, 512), "b3456": (6, 128, 3456)}   # dir: (blocks, channels, batch)


def means(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path, newline="")):
        if r["Counter_Name"] == counter and "board16_tower" in r["Kernel_Name"]:
            acc["board16_tower"].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def algorithmic(blocks, ch, B):
    pad_in, interior, w = B * 289 * ch * 4, B * 225 * ch * 4, 9 * ch * ch * 4
    return 2 * blocks * (pad_in + interior + w) + blocks * interior


def main():
    root, tag = sys.argv[1], sys.argv[2]
    path = os.path.join(REPO, "profiles", "conv_traffic.json")
    cur = json.load(open(path))
    recs = cur["records"] if "records" in cur else [cur]
    new = []
    for d, (blocks, ch, B) in TAGS.items():
        base = os.path.join(root, d)
        if not os.path.isdir(base):
            continue
        fetch = means(os.path.join(base, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
        write = means(os.path.join(base, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
        mp = os.path.join(base, "pmc_SQ_VALU_MFMA_BUSY_CYCLES_GRBM_GUI_ACTIVE", "run_counter_collection.csv")
        mf, gr = means(mp, "SQ_VALU_MFMA_BUSY_CYCLES"), means(mp, "GRBM_GUI_ACTIVE")
        k = "board16_tower"
        if k not in fetch:
            continue
        f, w = fetch[k] * 2 * 1024, write.get(k, 0.0) * 1024
        alg = algorithmic(blocks, ch, B)
        rec = {"kernel": "board16", "shape": "board16_tower", "config": f"{blocks}x{ch}_B{B}", "tag": tag,
               "boards_per_launch": B, "convs_per_launch": 2 * blocks,
               "hbm_bytes_per_launch": round(f + w), "fetch_bytes": round(f), "write_bytes": round(w),
               "algorithmic_bytes": alg, "traffic_over_algorithmic": round((f + w) / alg, 3)}
        if k in mf and k in gr:
            rec["mfma_busy"] = round(mf[k] * 8 / (4 * 256 * gr[k]), 4)
        new.append(rec)
        print(json.dumps(rec))
    keys = {(r["config"], r["shape"]) for r in new}
    recs = [r for r in recs if (r.get("config"), r.get("shape")) not in keys] + new
    json.dump({"records": recs}, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
