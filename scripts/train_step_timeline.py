"""Kernel-by-kernel timeline of one train step from a rocprofv3 kernel trace of
scripts/bench_train.py: every kernel of the median-length pipelined step with its
queue, start and duration relative to the step start, and per queue the gaps longer
than --gap us (where the stream waited on nothing it ran).

    python scripts/train_step_timeline.py TRACE.csv [--steps 10] [--gap 2]
"""
import argparse
import csv
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--gap", type=float, default=2.0)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "stem_mfma" in r["Kernel_Name"]]
sel = list(range(len(starts) - 2 * a.steps, len(starts) - a.steps - 1))
lens = [(int(rows[starts[si + 1]]["Start_Timestamp"]) - int(rows[starts[si]]["Start_Timestamp"]), si) for si in sel]
lens.sort()
_, si = lens[len(lens) // 2]
i0, i1 = starts[si], starts[si + 1]
t0 = int(rows[i0]["Start_Timestamp"])


def short(n):
    n = n.replace("void ", "").replace("azg::", "")
    return n.split("(")[0][:60]


print(f"median step {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us ({len(sel)} steps)")
last_end = {}
for r in rows[i0:i1]:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    mark = f"  gap {gap:6.1f}" if gap > a.gap else ""
    print(f"q{q:>3} {s / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {short(r['Kernel_Name'])}{mark}")
    last_end[q] = max(e, last_end.get(q, 0))
