#!/bin/bash
# Round 3 lease h: train GPU tests (head-chain stages, key 28) and the train-step A/B of
# the fused head stages.
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -12; [ $s -le 1 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "28=0;28=1;28=4;28=5;28=7" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
echo done
