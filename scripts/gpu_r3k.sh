#!/bin/bash
# Round 3 lease k: 8-wave weight-grad tile (key 16 = 4) -- bitwise key test and the
# train-step A/B against the 4-wave tile, plus the serial schedule's per-kernel times.
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 120 --timeout-method thread -k "schedule_keys and 16" > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -5; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "16=3;16=4;16=3,12=1;16=4,12=1" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr_serial4 -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 --serial --tune 16=4 > $O/tr_serial4.log 2>&1
s=$?; echo "serial trace rc $s"; [ $s -eq 0 ] || exit $s
echo done
