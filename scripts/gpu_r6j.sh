#!/bin/bash
# Round 6: split-fp16 dgrad (key 50) -- the train tests and an in-process train-step A/B
# of key 50 = 0 / 1 / 2 (-> gpurun_out/r6j)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6j
mkdir -p $O
AZG_TEST_TUNE=50=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1; t=$?
[ $t -eq 124 ] || [ $t -eq 137 ] || [ $t -eq 134 ] || [ $t -eq 139 ] && exit $t
timeout -k 10 300 python -u scripts/train_ab.py --variant 50=0 --variant 50=1 --variant 50=2 --no-bitwise --rounds 4 --steps 20 > $O/train_ab.log 2>&1
