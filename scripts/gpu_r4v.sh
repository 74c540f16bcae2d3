#!/bin/bash
# Round 4 lease v: head weight grads moved ahead of the tower backward -- train tests,
# bitwise vs round 3's library, step time vs the previous product library in one lease.
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; tail -1 $O/pytest.log; [ $s -eq 0 ] || exit $s
AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/ref.npz > $O/cmp_ref.log 2>&1 || exit 1
timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/new.npz > $O/cmp_new.log 2>&1 || exit 1
python scripts/train_lib_compare.py --compare /tmp/ref.npz /tmp/new.npz | tail -1
for i in 1 2 3; do
  timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "27=0" > $O/new$i.log 2>&1 || exit 1
  AZG_PV_LIB=scripts/_ref/libazg_pv_r4pre.so timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "27=0" > $O/pre$i.log 2>&1 || exit 1
  echo "new: $(tail -1 $O/new$i.log | cut -c50-100)   pre: $(tail -1 $O/pre$i.log | cut -c50-100)"
done
echo done
