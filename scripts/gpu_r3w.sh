#!/bin/bash
# Round 3 lease w: forward train-conv duration vs tile count (B = 112 / 128 / 145 / 146:
# 394 / 450 / 510 / 514 128x64 tiles on 512 two-per-CU slots) -- is the forward
# slot-quantization bound (the case for a stream-K forward)?
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for b in 112 128 145 146; do
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/b$b -o run -- python3 scripts/bench_train.py --steps 6 --warmup 2 --cpu-steps 0 --batch $b > $O/b$b.log 2>&1
  s=$?; echo "trace b$b rc $s"; [ $s -eq 0 ] || exit $s
done
python3 - <<'PY'
import csv, statistics, collections
for b in (112, 128, 145, 146):
    rows = list(csv.DictReader(open(f"gpurun_out/r3w/b{b}/run_kernel_trace.csv")))
    d = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if "conv3x3_train<" in n:
            key = n.split("(")[0].replace("void azg::conv3x3_train", "")
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    out = {k: round(statistics.median(v), 1) for k, v in sorted(d.items())}
    print(b, "tiles", 2 * ((b * 225 + 127) // 128), out)
PY
echo done
