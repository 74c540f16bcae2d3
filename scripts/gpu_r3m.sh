#!/bin/bash
# Round 3 lease m: train GPU tests on the new defaults (head chain 28, per-conv dZ), the
# weight-grad split sweep (key 27) and the serial / pipelined kernel traces.
set -o pipefail
O=gpurun_out/r3m
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_distributed.py -m gpu -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --splits 0,48,40,32,24 --ab "36=1;36=0;30=0,36=0" > $O/splits.log 2>&1
s=$?; tail -1 $O/splits.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; tail -c 400 $O/tr.log; [ $s -eq 0 ] || exit $s
echo done
