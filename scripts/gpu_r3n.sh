#!/bin/bash
# Round 3 lease n: 64x64 weight-grad tiles over fewer splits (key 16 = 5) -- oracle
# tests, bitwise schedule keys, A/B of the train step and a kernel trace.
set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 200 --timeout-method thread -k "split_variants or schedule_keys" > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "16=3;16=5;16=5,27=16;16=5,27=32;32=0" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr5 -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 --tune 16=5 > $O/tr5.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
echo done
