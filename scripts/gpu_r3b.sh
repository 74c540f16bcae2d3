#!/bin/bash
# Round 3 lease b: study-build bitwise tower variants, tower A/B (hand-off forms),
# train-step probe (key 24 / 25, host enqueue, graph floor), hand-off PMC A/B, and a
# kernel trace of the pipelined train step for its timeline.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
STUDY=alphazero-gomoku_amd/libazg_pv_study.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -v -k "schedule_keys" --timeout 240 --timeout-method thread > $O/pytest_keys.log 2>&1
s=$?; echo "keys rc $s"; tail -3 $O/pytest_keys.log; [ $s -le 1 ] || exit $s
AZG_PV_LIB=$STUDY timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -m gpu -v -k "tower" --timeout 240 --timeout-method thread > $O/pytest_study.log 2>&1
s=$?; echo "study pytest rc $s"; tail -5 $O/pytest_study.log; [ $s -le 1 ] || exit $s
AZG_PV_LIB=$STUDY timeout -k 10 400 python -u scripts/tower_r3_ab.py > $O/tower_ab.log 2>&1 || { echo "tower ab failed"; tail -30 $O/tower_ab.log; exit 1; }
grep batch $O/tower_ab.log
timeout -k 10 200 python -u scripts/train_r3_probe.py > $O/train_probe.log 2>&1 || { echo "train probe failed"; tail -30 $O/train_probe.log; exit 1; }
tail -1 $O/train_probe.log
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/train_trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/train_trace.log 2>&1 || { echo "train trace failed"; tail -20 $O/train_trace.log; exit 1; }
timeout -k 10 600 bash scripts/gpu_pmc_handoff_ab.sh > $O/pmc_handoff.log 2>&1 || { echo "pmc handoff failed"; tail -20 $O/pmc_handoff.log; exit 1; }
cat $O/pmc_handoff.log
echo done
