#!/bin/bash
# Round 4 lease p: board-keyed halo body (VAR 33) for the prologue-free train convs
# (key 50 = 33: every dgrad; the forward convs at C = 256) -- bitwise and step time at
# 6x128 and 10x256, B = 128.
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/a.npz > $O/cmp0.log 2>&1 || exit 1
timeout -k 10 300 python scripts/train_lib_compare.py --tune 50=33 --out /tmp/b.npz > $O/cmp1.log 2>&1 || exit 1
echo "50=33 vs 32: $(python scripts/train_lib_compare.py --compare /tmp/a.npz /tmp/b.npz | tail -1)"
for i in 1 2; do
  timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "50=32;50=33" > $O/p128_$i.log 2>&1 || exit 1
  tail -1 $O/p128_$i.log | cut -c1-150
done
for i in 1 2; do
  timeout -k 10 400 python -u scripts/train_r3_probe.py --blocks 10 --channels 256 --steps 10 --ab "50=32;50=33" > $O/p256_$i.log 2>&1 || exit 1
  tail -1 $O/p256_$i.log | cut -c1-150
done
echo done
