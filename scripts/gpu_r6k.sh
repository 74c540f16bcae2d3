#!/bin/bash
# Round 6: train-step kernel timeline (rocprofv3 kernel trace of scripts/bench_train.py)
# and the split-fp16 dgrad study's numbers under key 50 = 0 / 2 (-> gpurun_out/r6k)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/trace.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1 || exit 1
