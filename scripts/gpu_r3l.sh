#!/bin/bash
# Round 3 lease l: tiled head-FC stages (key 28 bit 3) -- oracle tests of every head
# chain variant, the train-step A/B, and a kernel trace with the new stages.
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 200 --timeout-method thread -k "schedule_keys and (33 or 34)" > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "28=4,34=0;28=28,34=0;28=28;28=4" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr28 -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 --tune 28=28 > $O/tr28.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
echo done
