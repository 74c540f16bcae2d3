"""HBM bytes per launch of the persistent residual tower from the PMC passes of
scripts/gpu_pmc_r3.sh -> "tower" records in profiles/conv_traffic.json (records of
other kernels / configs are kept; a record with the same config and shape is
replaced).  gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE x2 (wide
coalesced reads are tallied at half their bytes), KiB -> bytes.  Algorithmic bytes
per launch: every conv reads its padded input once (B x 289 x C x 4) and its weights
(9 C^2 x 4) and writes its interior output (B x 225 x C x 4); every second conv also
reads the residual (B x 225 x C x 4).

    python scripts/summarize_pmc_r3.py gpurun_out/pmc_r3 r3
"""
import collections
import csv
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAGS = {   # dir: (blocks, channels, batch)
    "t_b3456": (6, 128, 3456),
    "t_b512": (6, 128, 512),
    "t_256_b512": (10, 256, 512),
}


def means(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path, newline="")):
        if r["Counter_Name"] == counter and "conv_tower<" in r["Kernel_Name"]:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
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
        for k in fetch:
            f, w = fetch[k] * 2 * 1024, write.get(k, 0.0) * 1024
            alg = algorithmic(blocks, ch, B)
            shape = re.search(r"conv_tower<([^>]*)>", k).group(1)
            rec = {"kernel": "tower", "shape": f"conv_tower<{shape}>", "config": f"{blocks}x{ch}_B{B}", "tag": tag,
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
