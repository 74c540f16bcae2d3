#!/bin/bash
# Round 3 lease j: train-step kernel traces on the current product library (default
# two-stream schedule and the serial schedule, key 12 = 1), the head-chain A/B (key 28)
# and the per-layer eval conv at B = 128 for comparison with the train conv.
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr_default -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr_default.log 2>&1
s=$?; echo "default trace rc $s"; tail -c 600 $O/tr_default.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr_serial -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 --serial > $O/tr_serial.log 2>&1
s=$?; echo "serial trace rc $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "28=4;28=7;28=0;28=5;28=6" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/conv128 -o run -- python3 scripts/conv_probe.py --batch 128 --tower 0 --steps 20 > $O/conv128.log 2>&1
s=$?; echo "conv128 rc $s"; [ $s -eq 0 ] || exit $s
echo done
