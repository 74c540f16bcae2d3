#!/bin/bash
# Round 3 lease y: stream-K forward (key 44 = 1) vs its kernel at one tile per workgroup
# (2) vs conv3x3_train (0): bitwise keys + sum-order variants, train-step A/B, trace.
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v -k "schedule_keys or sum_order" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "44=0;44=2;44=1;44=0;44=2" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_trace_segments.py $O/tr/run_kernel_trace.csv
echo done
