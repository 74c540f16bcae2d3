#!/bin/bash
# Round 3 lease u: BN-backward fold with z by LDS-DMA (key 40 = 2) and the per-group
# fragment-address remat of the prologue train convs (no spills):
# bitwise key test + oracle gradients, train-step A/B, trace segments.
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 400 --timeout-method thread -k "schedule_keys or gradients_match or sum_order" > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "40=2;40=0;40=2;40=0" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_trace_segments.py $O/tr/run_kernel_trace.csv
echo done
