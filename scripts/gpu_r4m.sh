#!/bin/bash
# Round 4 lease m: bn_bwd_apply float4 per thread (key 49 = 1 / 2 / 4) with the float4
# slab reduction (key 48 = 1, now default): bitwise and step time.
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/a.npz > $O/cmp0.log 2>&1 || exit 1
for v in 1 2 4; do
  timeout -k 10 300 python scripts/train_lib_compare.py --tune 49=$v --out /tmp/b$v.npz > $O/cmp$v.log 2>&1 || exit 1
  echo "49=$v vs r3: $(python scripts/train_lib_compare.py --compare /tmp/a.npz /tmp/b$v.npz | tail -1)"
done
for i in 1 2; do
  timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "49=4;49=2;49=1;48=0" > $O/probe$i.log 2>&1 || exit 1
  tail -1 $O/probe$i.log | cut -c1-240
done
echo done
