#!/bin/bash
# Train-path check: GPU train tests + train-step timing (overlapped and serial).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tq
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tq/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/tq/pytest.log
[ $s -eq 0 ] || exit $s
timeout -k 10 200 python3 scripts/bench_train.py --steps 30 --cpu-steps 0 ${TRAIN_ARGS} 2>&1 | grep -v amdgpu.ids | tail -2
s=$?; [ $s -eq 0 ] || exit $s
timeout -k 10 200 python3 scripts/bench_train.py --steps 30 --cpu-steps 0 --serial ${TRAIN_ARGS} 2>&1 | grep -v amdgpu.ids | tail -2
