"""Condense a rocprofv3 run of bench.py (scripts/gpu_profile.sh output under
gpurun_out/prof_<TAG>/) into the committed evidence under profiles/:

  profiles/<TAG>_kernel_stats.csv   the --kernel-trace --stats summary, verbatim
  profiles/<TAG>_pmc.csv            per-kernel averages of every PMC pass
  profiles/<TAG>_summary.md         top kernels + the dominant conv kernel's HBM bytes
                                    (FETCH_SIZE x2 and WRITE_SIZE, KiB -> bytes, per the
                                    MI355X guide's gfx950 correction), MFMA busy and clock
  profiles/conv_traffic.json        per-launch HBM bytes of the tuned conv, read by bench.py

    python scripts/summarize_profile.py gpurun_out/prof_r1 r1 [--train gpurun_out/prof_r1_train]
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
BATCH, BLOCKS, CHANNELS = 512, 6, 128
FLOP_CONV = 2 * 225 * CHANNELS * 9 * CHANNELS   # per board per conv


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name, n=70):
    return name if len(name) <= n else name[:n] + "..."


def pmc_table(prof_dir):
    """{kernel_name: {counter: (mean, n)}} over all PMC passes."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(prof_dir, "pmc_*", "run_counter_collection.csv")):
        for row in read_csv(path):
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: (sum(v) / len(v), len(v)) for c, v in d.items()} for k, d in acc.items()}


def hbm_models(B, C=CHANNELS, n_params=1_892_650, S_wgrad=None):
    """Algorithmic HBM bytes per launch of the bandwidth-bound kernels (name prefix
    -> bytes) at batch B: every tensor read or written once, fp32."""
    M = B * 225
    act = M * C * 4
    m = {
        "azg::col_stats_kernel": act,
        "azg::bn_apply_kernel<128, false>": 2 * act,
        "azg::bn_apply_kernel<128, true>": 3 * act,
        "azg::bn_bwd_reduce_kernel": 3 * act,
        "azg::bn_bwd_apply_kernel<128, false>": 4 * act,
        "azg::bn_bwd_apply_kernel<128, true>": 5 * act,
        "azg::adam_kernel": 8 * 4 * n_params,
        "azg::grad_sqsum_kernel": 4 * n_params,
        "azg::heads_project<128, false>": act + 3 * M * 4,
        "azg::heads_project<128, true>": act + 3 * M * 4,
    }
    if S_wgrad:
        m["azg::wgrad_reduce_kernel"] = (S_wgrad + 1) * 9 * C * C * 4
    return m


def bw_table(stats, models):
    rows = []
    for r in stats:
        name = r["Name"]
        short_name = name.replace("void ", "")
        for k, b in models.items():
            if short_name.startswith(k):
                us = float(r["AverageNs"]) / 1e3
                rows.append(f"| `{short(short_name, 60)}` | {r['Calls']} | {us:.1f} | {b / 1e6:.1f} | "
                            f"{b / (us * 1e-6) / 1e9:.0f} | {b / (us * 1e-6) / 8e12 * 100:.0f} % |")
                break
    if not rows:
        return []
    return ["| HBM-bound kernel | calls | avg us | algorithmic MB | GB/s | of 8 TB/s |",
            "|---|---|---|---|---|---|"] + rows + [""]


def selfplay_busy(trace_csv):
    """GPU busy fraction over the self-play leg: union of kernel intervals between
    the first board-input stem kernel and the last kernel of the run."""
    rows = read_csv(trace_csv)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [a for a, _, n in iv if "stem_conv" in n and "true>" in n]
    if not starts:
        return None
    # the timed leg starts after the warm-up game: take the window from the last
    # gap > 50 ms before the final board-input stem launches
    t0 = starts[0]
    sel = [(a, b) for a, b, _ in iv if a >= t0]
    t_end = max(b for _, b in sel)
    busy, cur_a, cur_b = 0, None, None
    for a, b in sel:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    busy += cur_b - cur_a
    return {"window_ms": (t_end - t0) / 1e6, "busy_ms": busy / 1e6, "busy_frac": busy / max(t_end - t0, 1),
            "kernels": len(sel)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--train", default=None)
    ap.add_argument("--selfplay", default=None)
    args = ap.parse_args()
    os.makedirs(PROF, exist_ok=True)
    stats_path = os.path.join(args.prof_dir, "trace", "run_kernel_stats.csv")
    stats = read_csv(stats_path)
    shutil.copy(stats_path, os.path.join(PROF, f"{args.tag}_kernel_stats.csv"))
    pmc = pmc_table(args.prof_dir)
    with open(os.path.join(PROF, f"{args.tag}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "counter", "mean_per_dispatch", "dispatches"])
        for k in sorted(pmc):
            for c, (m, n) in sorted(pmc[k].items()):
                w.writerow([k, c, m, n])

    # dominant conv: the persistent residual tower when the forward used it (one
    # launch = all 2*BLOCKS convs), else the product-path per-layer conv kernels (the
    # most-called conv3x3 names: autotuning dispatches every candidate shape only twice)
    towers = [r for r in stats if "conv_tower" in r["Name"]]
    if towers:
        towers.sort(key=lambda r: int(r["Calls"]), reverse=True)
        tuned = towers[:1]
        convs_per_launch = 2 * BLOCKS
    else:
        convs = [r for r in stats if "conv3x3_halo" in r["Name"] or "conv3x3_mfma" in r["Name"]]
        convs.sort(key=lambda r: int(r["Calls"]), reverse=True)
        top_calls = int(convs[0]["Calls"]) if convs else 0
        tuned = [r for r in convs if int(r["Calls"]) >= top_calls // 2]
        convs_per_launch = 1
    calls = sum(int(r["Calls"]) for r in tuned)
    avg_ns = sum(float(r["TotalDurationNs"]) for r in tuned) / max(calls, 1)
    fetch = write = mfma = grbm = 0.0
    nk = 0
    for r in tuned:
        d = pmc.get(r["Name"], {})
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            wgt = int(r["Calls"])
            fetch += d["FETCH_SIZE"][0] * wgt
            write += d["WRITE_SIZE"][0] * wgt
            mfma += d.get("SQ_VALU_MFMA_BUSY_CYCLES", (0, 0))[0] * wgt
            grbm += d.get("GRBM_GUI_ACTIVE", (0, 0))[0] * wgt
            nk += wgt
    lines = [f"# rocprofv3 summary `{args.tag}` (bench.py: 6x128, B={BATCH} forward)", ""]
    lines.append("Source: `rocprofv3 --kernel-trace --stats` + separate `--pmc` passes "
                 "(scripts/gpu_profile.sh); raw files in this directory.")
    lines.append("")
    lines.append("| kernel | calls | avg us | total ms | % |")
    lines.append("|---|---|---|---|---|")
    for r in sorted(stats, key=lambda r: float(r["TotalDurationNs"]), reverse=True)[:14]:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
    lines.append("")
    traffic = None
    if nk:
        fetch_b = fetch / nk * 1024 * 2      # KiB, gfx950 streaming-read correction x2
        write_b = write / nk * 1024
        traffic = fetch_b + write_b
        in_b = BATCH * 289 * CHANNELS * 4 + 9 * CHANNELS * CHANNELS * 4
        out_b = BATCH * 225 * CHANNELS * 4
        # per conv: padded input once + weights + output; conv2 of each block also
        # reads the residual
        alg = convs_per_launch * (in_b + out_b + 0.5 * out_b)
        clk = grbm / nk / 8 / (avg_ns * 1e-9) / 1e9 if avg_ns else 0.0
        busy = mfma / nk / (4 * 256) / (grbm / nk / 8) if grbm else 0.0
        tflops = FLOP_CONV * BATCH * convs_per_launch / (avg_ns * 1e-9) / 1e12
        what = (f"persistent residual tower ({convs_per_launch} convs per launch)" if towers
                else "3x3 conv (tuned shape)")
        lines += [
            f"## Dominant kernel: {what}",
            "",
            f"* kernels: {', '.join('`' + short(r['Name'], 60) + '`' for r in tuned)}",
            f"* dispatches: {calls}, average duration {avg_ns / 1e3:.1f} us -> {tflops:.1f} TFLOP/s "
            f"({tflops / 157.3 * 100:.1f} % of the 157.3 TFLOP/s dense fp32 MFMA peak)",
            f"* HBM-side bytes per launch: FETCH_SIZE x2 = {fetch_b / 1e6:.1f} MB, WRITE_SIZE = {write_b / 1e6:.1f} MB, "
            f"total {traffic / 1e6:.1f} MB (algorithmic {alg / 1e6:.1f} MB: per conv padded input once + "
            "weights + output, + residual on every second conv)",
            f"* SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMD x 256 CU x GRBM_GUI_ACTIVE/8) = {busy * 100:.1f} %, "
            f"clock ~ {clk:.2f} GHz",
            "",
        ]
        rec = {"config": f"{BLOCKS}x{CHANNELS}_B{BATCH}", "tag": args.tag, "boards_per_launch": BATCH,
               "kernel": "tower" if towers else "conv3x3", "convs_per_launch": convs_per_launch,
               "hbm_bytes_per_launch": round(traffic), "fetch_bytes": round(fetch_b),
               "write_bytes": round(write_b), "algorithmic_bytes": round(alg),
               "traffic_over_algorithmic": round(traffic / alg, 3), "avg_launch_us": round(avg_ns / 1e3, 2)}
        path = os.path.join(PROF, "conv_traffic.json")
        old = json.load(open(path)) if os.path.exists(path) else {"records": []}
        recs = [r for r in old.get("records", [old]) if (r.get("kernel"), r.get("config")) != (rec["kernel"], rec["config"])]
        with open(path, "w") as f:
            json.dump({"records": recs + [rec]}, f, indent=1)
    lines += ["## HBM-bound kernels of the forward (B=512)", ""] + bw_table(stats, hbm_models(BATCH))
    if args.train:
        tpath = os.path.join(args.train, "trace", "run_kernel_stats.csv")
        if os.path.exists(tpath):
            shutil.copy(tpath, os.path.join(PROF, f"{args.tag}_train_kernel_stats.csv"))
            ts = read_csv(tpath)
            lines += ["## Train step (scripts/bench_train.py: 6x128, B=128)", "",
                      "| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
            for r in sorted(ts, key=lambda r: float(r["TotalDurationNs"]), reverse=True)[:16]:
                lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                             f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
            lines.append("")
            lines += ["### HBM-bound kernels of the train step (B=128)", ""]
            lines += bw_table(ts, hbm_models(128, S_wgrad=(128 * 225 + 543) // 544))
    if args.selfplay:
        tr = os.path.join(args.selfplay, "trace", "run_kernel_trace.csv")
        st = os.path.join(args.selfplay, "trace", "run_kernel_stats.csv")
        if os.path.exists(tr):
            shutil.copy(st, os.path.join(PROF, f"{args.tag}_selfplay_kernel_stats.csv"))
            b = selfplay_busy(tr)
            if b:
                lines += ["## Self-play leg (bench.py: 256 games x 400 sims, native search, int8 leaves)", "",
                          f"* GPU busy {b['busy_ms']:.1f} ms of {b['window_ms']:.1f} ms "
                          f"({b['busy_frac'] * 100:.1f} %) from the first board-input forward to the last "
                          f"kernel ({b['kernels']} kernels; includes the warm-up game and bucket warm-up)", ""]
    with open(os.path.join(PROF, f"{args.tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
