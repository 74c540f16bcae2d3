"""Per-step timeline of a rocprofv3 kernel trace: kernel start offsets, durations,
queue, and the idle gaps of the merged busy intervals.

    python scripts/trace_timeline.py TRACE.csv [--marker stem_mfma] [--step -5] [--quiet]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="stem_mfma")
ap.add_argument("--step", type=int, default=-5)
ap.add_argument("--quiet", action="store_true")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
i0, i1 = starts[a.step - 1], starts[a.step]
st = rows[i0:i1]
t0, tend = int(st[0]["Start_Timestamp"]), int(rows[i1]["Start_Timestamp"])
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70], r["Queue_Id"]) for r in st)
busy, gaps = 0, 0.0
cs, ce = iv[0][0], iv[0][1]
for s, e, _, _ in iv[1:]:
    if s > ce:
        gaps += s - ce
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
by = {}
for s, e, n, q in iv:
    k = n.split("(")[0]
    d = by.setdefault(k, [0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1e3
print(f"step span {(tend - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {gaps / 1e3:.1f} us, kernels {len(iv)}")
for k, (n, us) in sorted(by.items(), key=lambda x: -x[1][1]):
    print(f"  {us:8.1f} us {n:4d}x  {k}")
if not a.quiet:
    for s, e, n, q in iv:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n}")
