"""Round-4 train-conv PMC table (scripts/gpu_r4_pmc_train.sh) -> profiles/<tag>_train_pmc.md.

Per kernel of the 6x128, B = 128 train step: launches per step, mean duration (kernel
trace of the same command), scratch bytes per lane, MFMA fraction of the fp32 peak
(algorithmic FLOP / duration), SQ MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over
4 SIMD x 256 CU x GRBM_GUI_ACTIVE / 8), VALU / MFMA instructions, LDS bank-conflict
cycles, SQ_WAIT_ANY share of wave cycles, and HBM bytes (FETCH_SIZE x2 + WRITE_SIZE,
the gfx950 corrections of MI355X_MICROARCH.md) against the algorithmic bytes; then the
conv durations with the fused BN apply (key 23 = 0) and fused finalize (key 24 = 0)
switched off.

    python scripts/summarize_train_pmc_r4.py gpurun_out/pmc_train_r4 r4
"""
import collections
import csv
import glob
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, C = 128, 128
M = B * 225
CONV_FLOP = 2 * M * 9 * C * C
ACT, PAD = M * C * 4, B * 289 * C * 4
W = 9 * C * C * 4
STEPS = 10
ALG = {   # algorithmic HBM bytes per launch
    # forward, BN apply in the staging: read raw z (+ residual) and write a's own rows + z
    "conv3x3_train<128, 2, 1, true, 1": PAD + W + ACT + ACT,
    "conv3x3_train<128, 2, 1, true, 2": 2 * PAD + W + ACT + ACT,
    # dgrad: read dZ, act, z (BN-backward sums), (+ the residual gradient), write out
    "conv3x3_train<128, 2, 2, true, 0": PAD + W + 2 * ACT + ACT,
    "conv3x3_train<128, 3, 2, true, 0": PAD + W + 3 * ACT + ACT,
    "conv3x3_wgrad_nat<128>": 2 * ACT + 56 * W,
}


def short(n):
    return n.replace("void ", "").replace("azg::", "").split("(")[0]


def trace_stats(d):
    f = glob.glob(os.path.join(d, "**", "run_kernel_trace.csv"), recursive=True)[0]
    dur, scr = collections.defaultdict(list), {}
    for r in csv.DictReader(open(f, newline="")):
        k = short(r["Kernel_Name"])
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        scr[k] = int(r.get("Scratch_Size", 0) or 0)
    return dur, scr


def main():
    base, tag = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(base, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur, scr = trace_stats(os.path.join(base, "tr_default"))
    mean = lambda k, c: statistics.mean(acc[k][c]) if acc[k].get(c) else None
    rows = []
    for k, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        if not any(s in k for s in ("conv3x3_train", "wgrad", "bn_bwd_apply", "bn_apply")):
            continue
        d = statistics.median(ds)
        per = len(ds) / (STEPS + 8)   # bench_train: warmup 3 + 3 timed loops of `steps`... approximate
        mf = CONV_FLOP / (d * 1e-6) / 157.3e12 if ("conv3x3" in k) else None
        busy = mean(k, "SQ_VALU_MFMA_BUSY_CYCLES")
        gui = mean(k, "GRBM_GUI_ACTIVE")
        sqb = busy / (4 * 256 * gui / 8) if busy is not None and gui else None
        valu, mfma = mean(k, "SQ_INSTS_VALU"), mean(k, "SQ_INSTS_MFMA")
        wait, cyc = mean(k, "SQ_WAIT_ANY"), mean(k, "SQ_WAVE_CYCLES")
        fetch, write = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
        hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        alg = next((v for p, v in ALG.items() if k.startswith(p)), None)
        rows.append((k, d, scr.get(k, 0), mf, sqb, (valu / mfma) if valu and mfma else None,
                     mean(k, "SQ_LDS_BANK_CONFLICT"), (wait / cyc) if wait and cyc else None, hbm, alg))
    out = [f"# Train-step PMC ({tag}): 6x128, B = 128, product schedule", "",
           "`scripts/gpu_r4_pmc_train.sh` (rocprofv3 --pmc passes, one counter group each, over "
           "`scripts/bench_train.py`; counter collection serialises the kernels) and a kernel trace of the same "
           "command for the durations and scratch.  MFMA frac = 2*M*9*C^2 / duration / 157.3 TFLOP/s; SQ MFMA busy = "
           "SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMD x 256 CU x GRBM_GUI_ACTIVE / 8); HBM = FETCH_SIZE x2 + WRITE_SIZE (KiB, "
           "gfx950 corrections) per launch against the algorithmic bytes.", "",
           "| kernel | median us (in-step) | scratch B/lane | MFMA frac | SQ MFMA busy | VALU/MFMA | LDS conflict cycles | "
           "wait_any / wave cycles | HBM MB (alg.) |", "|---|---|---|---|---|---|---|---|---|"]
    f = lambda v, fmt: fmt.format(v) if v is not None else ""
    for k, d, sc, mf, sqb, vm, lds, wt, hbm, alg in rows:
        hb = f"{hbm / 1e6:.1f}" + (f" ({alg / 1e6:.1f})" if alg else "") if hbm is not None else ""
        out.append(f"| `{k}` | {d:.1f} | {sc} | {f(mf, '{:.1%}')} | {f(sqb, '{:.1%}')} | {f(vm, '{:.2f}')} | "
                   f"{f(lds, '{:.0f}')} | {f(wt, '{:.1%}')} | {hb} |")
    out += ["", "Conv durations (median in-step us) with the fused stages switched off:", "",
            "| kernel | default | key 23 = 0 (separate BN apply passes) | key 24 = 0 (separate finalize kernels) |",
            "|---|---|---|---|"]
    t23, _ = trace_stats(os.path.join(base, "tr_23_0"))
    t24, _ = trace_stats(os.path.join(base, "tr_24_0"))
    names = sorted(set(dur) | set(t23) | set(t24))
    for k in names:
        if "conv3x3_train" not in k and "bn_fin_tiles" not in k and "bn_apply" not in k:
            continue
        g = lambda t: f"{statistics.median(t[k]):.1f} x{len(t[k])}" if k in t else "-"
        out.append(f"| `{k}` | {g(dur)} | {g(t23)} | {g(t24)} |")
    path = os.path.join(REPO, "profiles", f"{tag}_train_pmc.md")
    open(path, "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
