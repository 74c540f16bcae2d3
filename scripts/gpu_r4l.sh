#!/bin/bash
# Round 4 lease l: float4 slab reduction (key 48 = 1 / 2) vs scalar: bitwise and step time.
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/a.npz > $O/cmp0.log 2>&1 || exit 1
for v in 1 2; do
  timeout -k 10 300 python scripts/train_lib_compare.py --tune 48=$v --out /tmp/b$v.npz > $O/cmp$v.log 2>&1 || exit 1
  echo "48=$v: $(python scripts/train_lib_compare.py --compare /tmp/a.npz /tmp/b$v.npz | tail -1)"
done
for i in 1 2; do
  timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "48=0;48=1;48=2" > $O/probe$i.log 2>&1 || exit 1
  tail -1 $O/probe$i.log | cut -c1-200
done
echo done
