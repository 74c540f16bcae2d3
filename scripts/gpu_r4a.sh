#!/bin/bash
# Round 4 lease a: the persistent train backward (key 43) against the round-3 library
# (bitwise, scripts/train_lib_compare.py), its GPU tests, and the train-step A/B.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python scripts/train_lib_compare.py --out $O/ref.npz > $O/cmp_ref.log 2>&1
s=$?; echo "ref rc $s"; tail -3 $O/cmp_ref.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python scripts/train_lib_compare.py --out $O/new.npz > $O/cmp_new.log 2>&1
s=$?; echo "new rc $s"; tail -3 $O/cmp_new.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python scripts/train_lib_compare.py --tune 43=0 --out $O/new0.npz > $O/cmp_new0.log 2>&1
s=$?; echo "new0 rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_lib_compare.py --compare $O/ref.npz $O/new.npz | tail -5
python scripts/train_lib_compare.py --compare $O/ref.npz $O/new0.npz | tail -3
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "bwd_tower or schedule_keys" > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -12; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "43=1;43=0" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
echo done
