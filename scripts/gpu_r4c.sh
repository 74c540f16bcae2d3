#!/bin/bash
# Round 4 lease c: the pruned product library's GPU tests (train, game-level oracle
# parity, distributed, tower claim queues), the persistent backward in the study build,
# the train step bitwise against round 3's library, the train-step kernel timeline and
# the A/B of the BN apply grid cap (key 44).
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_oracle_games.py tests/test_gpu_distributed.py "tests/test_gpu_forward.py::test_persistent_tower_bitwise_equals_per_layer_launches" -x -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "PASS|FAIL|ERROR|passed|failed|identical to the oracle|skipped" $O/pytest.log | tail -40; [ $s -eq 0 ] || exit $s
AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k bwd_tower > $O/pytest_study.log 2>&1
s=$?; echo "pytest study rc $s"; grep -E "passed|failed" $O/pytest_study.log | tail -3; [ $s -eq 0 ] || exit $s
AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/ref.npz > $O/cmp_ref.log 2>&1 || exit 1
timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/new.npz > $O/cmp_new.log 2>&1 || exit 1
python scripts/train_lib_compare.py --compare /tmp/ref.npz /tmp/new.npz | tail -4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_trace_segments.py $O/tr/run_kernel_trace.csv
python scripts/train_step_timeline.py $O/tr/run_kernel_trace.csv > $O/timeline.txt
head -3 $O/timeline.txt
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "44=0;44=256;44=512;44=1024;44=2048" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
echo done
