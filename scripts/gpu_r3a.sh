#!/bin/bash
# Round 3, first lease: GPU parity suite on the new tower hand-off forms, the study
# build's bitwise variant check, the tower A/B and the train-step probe.
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
export PYTHONUNBUFFERED=1
STUDY=alphazero-gomoku_amd/libazg_pv_study.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
AZG_PV_LIB=$STUDY timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -m gpu -x -v -k "tower" --timeout 240 --timeout-method thread > $O/pytest_study.log 2>&1 || { echo "study pytest failed"; tail -30 $O/pytest_study.log; exit 1; }
AZG_PV_LIB=$STUDY timeout -k 10 400 python -u scripts/tower_r3_ab.py > $O/tower_ab.log 2>&1 || { echo "tower ab failed"; tail -30 $O/tower_ab.log; exit 1; }
timeout -k 10 200 python -u scripts/train_r3_probe.py > $O/train_probe.log 2>&1 || { echo "train probe failed"; tail -30 $O/train_probe.log; exit 1; }
tail -3 $O/pytest.log; cat $O/tower_ab.log | grep batch; cat $O/train_probe.log | tail -2
