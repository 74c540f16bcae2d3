"""Round-3 rocprofv3 evidence -> profiles/:

  r3_selfplay_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the headline bench
                                 command (configs[2] self-play to game end), verbatim
  r3_forward_kernel_stats.csv    same for the configs[1] forward leg (B = 512)
  r3_train_kernel_stats.csv      same for scripts/bench_train.py (6x128, B = 128), if given
  r3_summary.md                  the residual-conv launches INSIDE the timed self-play
                                 window (trace timestamps; autotuning launches before it
                                 excluded) against the bench JSON's hipEvent totals and
                                 roofline; the forward leg's tower; the PMC traffic
                                 records (profiles/conv_traffic.json, tag r3); one train
                                 step's timeline

    python scripts/summarize_r3.py gpurun_out/r3c [gpurun_out/r3b/train_trace] [tag]
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
PEAK = 157.3e12


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def conv_flop(ch):
    return 2 * 225 * ch * 9 * ch


def window(trace, seconds, names):
    t_end = max(int(r["End_Timestamp"]) for r in trace)
    t0 = t_end - int(seconds * 1e9)
    by = {}
    for r in trace:
        if int(r["Start_Timestamp"]) >= t0 and any(n in r["Kernel_Name"] for n in names):
            k = r["Kernel_Name"].split("(")[0]
            d = by.setdefault(k, [0, 0.0])
            d[0] += 1
            d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return by


def main():
    root = sys.argv[1]
    train_dir = sys.argv[2] if len(sys.argv) > 2 else None
    tag = sys.argv[3] if len(sys.argv) > 3 else "r3"
    sp_dir, fw_dir = os.path.join(root, "sp", "trace"), os.path.join(root, "fwd", "trace")
    shutil.copy(os.path.join(sp_dir, "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_selfplay_kernel_stats.csv"))
    shutil.copy(os.path.join(fw_dir, "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_forward_kernel_stats.csv"))
    bench = json.loads(open(os.path.join(root, "sp", "bench.json")).read().strip().splitlines()[-1])
    sp, det, roof = bench["selfplay"], bench["selfplay"]["detail"], bench["roofline"]
    peak = roof.get("peak", PEAK / 1e12) * 1e12   # the instruction's roofline (split-fp16: F16 peak / 3)
    by = window(rows(os.path.join(sp_dir, "run_kernel_trace.csv")), sp["seconds"],
                ("conv_tower<128", "conv3x3_halo<128"))
    L = [f"# rocprofv3 evidence, {tag}", "",
         "## Headline: configs[2] self-play to game end", "",
         f"`rocprofv3 --kernel-trace --stats -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 "
         f"--big-steps 0` (scripts/{os.environ.get('AZG_TRACE_SCRIPT', f'gpu_{tag}k.sh')}): {bench['value']:.0f} leaf boards/s over {sp['seconds']:.1f} s, "
         f"{sp['rounds']} move rounds, games {det['game_length_rank0']} moves long, mean leaf batch "
         f"{det['mean_batch_rank0']}.", "",
         f"Residual-conv launches inside the timed window (the last {sp['seconds']:.1f} s of the trace; the "
         "autotuning launches before it excluded):", "",
         "| kernel | launches | device ms | avg us |", "|---|---|---|---|"]
    for k, (n, ms) in sorted(by.items(), key=lambda x: -x[1][1]):
        L.append(f"| `{k}` | {n} | {ms:.1f} | {ms / n * 1e3:.1f} |")
    tower = {k: v for k, v in by.items() if "conv_tower" in k}
    tn, tms = sum(v[0] for v in tower.values()), sum(v[1] for v in tower.values())
    ev_ms = det["kernel_ms_rank0"].get("tower", 0.0)
    ev_n = det["kernel_launches_rank0"].get("tower", 0)
    flop = roof["flop_per_launch"] * roof["launches"]
    L += ["",
          f"* Dominant kernel, the persistent tower: rocprofv3 {tn} launches, {tms:.1f} ms; the bench's own hipEvents "
          f"on the tower's stream: {ev_n} launches, {ev_ms:.1f} ms ({(tms - ev_ms) / ev_ms * 100:+.2f} %).",
          f"* Its roofline from the rocprofv3 time: {flop / 1e12:.1f} TFLOP / {tms / 1e3:.3f} s = "
          f"{flop / (tms / 1e3) / 1e12:.2f} TFLOP/s = {flop / (tms / 1e3) / peak * 100:.2f} % of {peak / 1e12:.1f} "
          f"(JSON `roofline.frac` {roof['frac'] * 100:.2f} %, from hipEvents).",
          f"* GPU busy {det['gpu_busy_share_rank0'] * 100:.1f} % of the wall time.", ""]
    # forward leg
    fb = json.loads(open(os.path.join(root, "fwd", "bench.json")).read().strip().splitlines()[-1])["forward_b512"]
    fr = rows(os.path.join(fw_dir, "run_kernel_trace.csv"))
    ft = [r for r in fr if "conv_tower<128" in r["Kernel_Name"]]
    ft = ft[-fb["steps"]:]
    if ft:
        us = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ft) / len(ft) / 1e3
        f512 = conv_flop(128) * 12 * 512
        L += ["## configs[1] forward, B = 512 (bench `forward_b512`)", "",
              f"* `{ft[-1]['Kernel_Name'].split('(')[0]}`: {len(ft)} timed launches, {us:.1f} us average = "
              f"{f512 / (us * 1e-6) / 1e12:.2f} TFLOP/s = {f512 / (us * 1e-6) / peak * 100:.2f} % of peak "
              f"(JSON: {fb['roofline']['avg_launch_us']} us, {fb['roofline']['frac'] * 100:.2f} %); "
              f"{fb['boards_per_s']:.0f} boards/s for the whole forward.", ""]
    # PMC records
    recs = [r for r in json.load(open(os.path.join(PROF, "conv_traffic.json")))["records"]
            if r.get("tag") == tag or (len(r.get("tag", "")) == len(tag) + 1 and r["tag"].startswith(tag))]
    if recs:
        L += ["## HBM traffic of the tower (PMC, scripts/gpu_pmc_r3.sh / gpu_pmc_r5.sh; FETCH_SIZE x2 + WRITE_SIZE)", "",
              "| kernel | config | HBM MB / launch | algorithmic MB | ratio | SQ MFMA busy |", "|---|---|---|---|---|---|"]
        for r in recs:
            L.append(f"| `{r['shape']}` | {r['config']} | {r['hbm_bytes_per_launch'] / 1e6:.0f} | "
                     f"{r['algorithmic_bytes'] / 1e6:.0f} | {r['traffic_over_algorithmic']} | "
                     f"{r.get('mfma_busy', 0) * 100:.1f} % |")
        L.append("")
    if train_dir:
        shutil.copy(os.path.join(train_dir, "run_kernel_stats.csv") if os.path.exists(
            os.path.join(train_dir, "run_kernel_stats.csv")) else os.path.join(train_dir, "run_kernel_trace.csv"),
            os.path.join(PROF, f"{tag}_train_kernel_trace.csv"))
        tt = sorted(rows(os.path.join(train_dir, "run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
        starts = [i for i, r in enumerate(tt) if "stem_mfma" in r["Kernel_Name"]]
        if len(starts) > 16:   # a step of the pipelined, un-instrumented loop of bench_train.py
            i0, i1 = starts[-15], starts[-14]
            st = tt[i0:i1]
            a = int(st[0]["Start_Timestamp"])
            b = int(tt[i1]["Start_Timestamp"])
            agg = {}
            for r in st:
                k = r["Kernel_Name"].split("(")[0]
                d = agg.setdefault(k, [0, 0.0])
                d[0] += 1
                d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            L += ["## Train step (scripts/bench_train.py: 6x128, B = 128, un-instrumented pipelined loop)", "",
                  f"One step spans {(b - a) / 1e3:.0f} us (two streams: weight grads on a low-priority side "
                  "stream).", "", "| kernel | per step | device us |", "|---|---|---|"]
            for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
                L.append(f"| `{k}` | {n} | {us:.0f} |")
            L.append("")
    open(os.path.join(PROF, f"{tag}_summary.md"), "w").write("\n".join(L) + "\n")
    print("\n".join(L))


if __name__ == "__main__":
    main()
