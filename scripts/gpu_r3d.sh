#!/bin/bash
# Round 3 lease d: GPU suite with the fused train head chain, and the train-step A/B
# of the head chain (key 28) on the product library.
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -12; [ $s -le 1 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "28=1;28=0" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/train_trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/train_trace.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
echo done
