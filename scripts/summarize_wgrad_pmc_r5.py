"""Round-5 weight-grad PMC table (scripts/gpu_r5_pmc_wgrad.sh) -> profiles/r5_wgrad_pmc.md.

Both weight-grad tile forms (key 48 = 0: round 4's conv3x3_wgrad_nat, 1: round 5's
conv3x3_wgrad_nat2) and their slab reductions, with the train convs beside them: the
columns of scripts/summarize_train_pmc_r4.py (median in-step duration from a kernel
trace, MFMA fraction, SQ MFMA busy, VALU / MFMA, LDS conflicts, SQ_WAIT_ANY share, HBM
bytes with the gfx950 corrections), and the train step's mean per-step time of each
trace run.

    python scripts/summarize_wgrad_pmc_r5.py gpurun_out/r5_pmc_wgrad
"""
import collections
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_train_pmc_r4 import ALG, CONV_FLOP, REPO, short, trace_stats  # noqa: E402

ALG = dict(ALG)
ALG["conv3x3_wgrad_nat2<128>"] = ALG["conv3x3_wgrad_nat<128>"]


def table(base):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(base, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur, scr = trace_stats(os.path.join(base, "tr_default"))
    mean = lambda k, c: statistics.mean(acc[k][c]) if acc[k].get(c) else None
    rows = []
    for k, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        if not any(s in k for s in ("conv3x3", "wgrad")):
            continue
        d = statistics.median(ds)
        mf = CONV_FLOP / (d * 1e-6) / 157.3e12 if "conv3x3" in k else None
        busy, gui = mean(k, "SQ_VALU_MFMA_BUSY_CYCLES"), mean(k, "GRBM_GUI_ACTIVE")
        sqb = busy / (4 * 256 * gui / 8) if busy is not None and gui else None
        valu, mfma = mean(k, "SQ_INSTS_VALU"), mean(k, "SQ_INSTS_MFMA")
        wait, cyc = mean(k, "SQ_WAIT_ANY"), mean(k, "SQ_WAVE_CYCLES")
        fetch, write = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
        hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        alg = next((v for p, v in ALG.items() if k.startswith(p)), None)
        rows.append((k, d, len(ds), scr.get(k, 0), mf, sqb, (valu / mfma) if valu and mfma else None,
                     mean(k, "SQ_LDS_BANK_CONFLICT"), (wait / cyc) if wait and cyc else None, hbm, alg))
    return rows


def main():
    base = sys.argv[1]
    f = lambda v, fmt: fmt.format(v) if v is not None else ""
    out = ["# Weight-grad tile, round 4 (v1) vs round 5 (v2): PMC + kernel trace (6x128, B = 128)", "",
           "`scripts/gpu_r5_pmc_wgrad.sh`: the round-4 train PMC passes over `scripts/bench_train.py --tune 48=v` "
           "(counter collection serialises the kernels) and a kernel trace of the same command.  v2 = padded-row "
           "table, buffer LDS-DMA, MFMA-layout slabs (pv_wgrad.h wgrad_nat_tile2); the slabs and dW are bitwise "
           "those of v1 (tests/test_gpu_train.py key 48; scripts/train_lib_compare.py against round 4's library).",
           ""]
    for v in ("1", "0"):
        d = os.path.join(base, f"v{v}")
        if not os.path.isdir(d):
            continue
        out += [f"## key 48 = {v} ({'v2, round 5' if v == '1' else 'v1, round 4'})", "",
                "| kernel | median us (in-step) | launches | scratch B/lane | MFMA frac | SQ MFMA busy | VALU/MFMA | "
                "LDS conflict cycles | wait_any / wave cycles | HBM MB (alg.) |",
                "|---|---|---|---|---|---|---|---|---|---|"]
        for k, dd, n, sc, mf, sqb, vm, lds, wt, hbm, alg in table(d):
            hb = f"{hbm / 1e6:.1f}" + (f" ({alg / 1e6:.1f})" if alg else "") if hbm is not None else ""
            out.append(f"| `{k}` | {dd:.1f} | {n} | {sc} | {f(mf, '{:.1%}')} | {f(sqb, '{:.1%}')} | {f(vm, '{:.2f}')} | "
                       f"{f(lds, '{:.0f}')} | {f(wt, '{:.1%}')} | {hb} |")
        out.append("")
    path = os.path.join(REPO, "profiles", "r5_wgrad_pmc.md")
    open(path, "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
