"""Per-segment durations of train steps in a rocprofv3 kernel trace of
scripts/bench_train.py: start (stem .. first residual conv), forward convs, heads
(last forward conv .. first dgrad conv), backward (first dgrad .. last dgrad end),
tail (.. next step's stem), median over the un-instrumented pipelined steps.

    python scripts/train_trace_segments.py TRACE.csv [--steps 10]
"""
import argparse
import csv
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=10, help="bench_train.py --steps (the pipelined loop)")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "stem_mfma" in r["Kernel_Name"]]
# bench_train.py: warmup, a synced loop, the pipelined loop, the instrumented loop
sel = range(len(starts) - 2 * a.steps, len(starts) - a.steps - 1)
seg = {k: [] for k in ("start", "forward", "heads", "backward", "tail", "step")}
for si in sel:
    i0, i1 = starts[si], starts[si + 1]
    st = rows[i0:i1]
    q = st[0]["Queue_Id"]
    t0, tn = int(st[0]["Start_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    conv = [r for r in st if "conv3x3_train" in r["Kernel_Name"]]
    fwd = [r for r in conv if ", 1, true," in r["Kernel_Name"] or ", 1, true, 2" in r["Kernel_Name"]]
    nf = len(conv) // 2
    fwd, bwd = conv[:nf], conv[nf:]
    seg["start"].append((int(fwd[0]["Start_Timestamp"]) - t0) / 1e3)
    seg["forward"].append((int(fwd[-1]["End_Timestamp"]) - int(fwd[0]["Start_Timestamp"])) / 1e3)
    seg["heads"].append((int(bwd[0]["Start_Timestamp"]) - int(fwd[-1]["End_Timestamp"])) / 1e3)
    seg["backward"].append((int(bwd[-1]["End_Timestamp"]) - int(bwd[0]["Start_Timestamp"])) / 1e3)
    seg["tail"].append((tn - int(bwd[-1]["End_Timestamp"])) / 1e3)
    seg["step"].append((tn - t0) / 1e3)
print({k: round(statistics.median(v), 1) for k, v in seg.items()}, f"({len(seg['step'])} steps)")
