"""Round-2 profile evidence (scripts/gpu_profile_r2.sh output) -> profiles/:

  r2_selfplay_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the headline bench
                                 command (self-play to game end), verbatim
  r2_train_kernel_stats.csv      same for scripts/bench_train.py (6x128, B=128)
  r2_selfplay_summary.md         the residual-conv launches INSIDE the timed self-play
                                 window (trace timestamps; autotuning launches before it
                                 excluded) against the bench JSON's hipEvent totals, and
                                 the train-step timeline of one step

    python scripts/summarize_r2.py gpurun_out/prof_r2 [tag]
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
FLOP_CONV = 2 * 225 * 128 * 9 * 128


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "prof_r2")
    tag = sys.argv[2] if len(sys.argv) > 2 else "r2"
    sp_dir, tr_dir = os.path.join(root, "sp", "trace"), os.path.join(root, "train", "trace")
    shutil.copy(os.path.join(sp_dir, "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_selfplay_kernel_stats.csv"))
    shutil.copy(os.path.join(tr_dir, "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_train_kernel_stats.csv"))
    bench = json.loads(open(os.path.join(root, "sp", "bench.json")).read().strip().splitlines()[-1])
    sp = bench["selfplay"]
    trace = rows(os.path.join(sp_dir, "run_kernel_trace.csv"))
    t_end = max(int(r["End_Timestamp"]) for r in trace)
    t0 = t_end - int(sp["seconds"] * 1e9)
    conv = [r for r in trace if int(r["Start_Timestamp"]) >= t0 and
            ("conv_tower<128" in r["Kernel_Name"] or "conv3x3_halo<128" in r["Kernel_Name"])]
    by = {}
    for r in conv:
        k = r["Kernel_Name"].split("(")[0]
        d = by.setdefault(k, [0, 0.0])
        d[0] += 1
        d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot_n = sum(v[0] for v in by.values())
    tot_ms = sum(v[1] for v in by.values())
    det = sp["detail"]
    ev_ms = det["kernel_ms_rank0"].get("tower", 0) + det["kernel_ms_rank0"].get("conv3x3", 0)
    ev_n = det["kernel_launches_rank0"].get("tower", 0) + det["kernel_launches_rank0"].get("conv3x3", 0)
    roof = bench["roofline"]
    L = [f"# rocprofv3 evidence, {tag}", "",
         "## Headline: configs[2] self-play to game end (bench.py, this command under rocprofv3)", "",
         f"`rocprofv3 --kernel-trace --stats -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 "
         f"--big-steps 0` (scripts/gpu_profile_r2.sh): {bench['value']:.0f} leaf boards/s over "
         f"{sp['seconds']:.1f} s, {sp['rounds']} move rounds, games {det['game_length_rank0']} moves long, "
         f"mean leaf batch {det['mean_batch_rank0']}.", "",
         "Residual-conv launches inside the timed window (the last "
         f"{sp['seconds']:.1f} s of the trace; the autotuning launches before it excluded):", "",
         "| kernel | launches | device ms | avg us |", "|---|---|---|---|"]
    for k, (n, ms) in sorted(by.items(), key=lambda x: -x[1][1]):
        L.append(f"| `{k}` | {n} | {ms:.1f} | {ms / n * 1e3:.1f} |")
    L += ["", f"* rocprofv3: {tot_n} launches, {tot_ms:.1f} ms of device time; the bench's own hipEvents "
              f"(JSON `selfplay.detail`): {ev_n} launches, {ev_ms:.1f} ms "
              f"({(tot_ms - ev_ms) / ev_ms * 100:+.1f} %).",
          f"* JSON roofline: {roof['achieved']} TFLOP/s = {roof['frac'] * 100:.1f} % of 157.3 (residual convs, "
          f"all launches in the run: {roof.get('all_residual_convs_frac', roof['frac']) * 100:.1f} %); "
          f"GPU busy {det['gpu_busy_share_rank0'] * 100:.1f} % of the wall time.", ""]
    # train step: one step's timeline
    tt = sorted(rows(os.path.join(tr_dir, "run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(tt) if "stem_mfma" in r["Kernel_Name"]]
    if len(starts) > 6:
        st = tt[starts[-6]:starts[-5]]
        a, b = int(st[0]["Start_Timestamp"]), int(tt[starts[-5]]["Start_Timestamp"])
        agg = {}
        for r in st:
            k = r["Kernel_Name"].split("(")[0]
            d = agg.setdefault(k, [0, 0.0])
            d[0] += 1
            d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        L += ["## Train step (scripts/bench_train.py: 6x128, B=128, rocprofv3 kernel trace)", "",
              f"One step spans {(b - a) / 1e3:.0f} us of device time (two streams: weight grads on a "
              "low-priority side stream).", "", "| kernel | per step | device us |", "|---|---|---|"]
        for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:16]:
            L.append(f"| `{k}` | {n} | {us:.0f} |")
        L.append("")
    open(os.path.join(PROF, f"{tag}_selfplay_summary.md"), "w").write("\n".join(L) + "\n")
    print("\n".join(L))


if __name__ == "__main__":
    main()
