#!/bin/bash
# train-step check: GPU train parity tests, then serial / overlapped step timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_train.log 2>&1
s=$?; echo "pytest train exit $s"; tail -15 gpurun_out/pytest_train.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 200 python3 scripts/bench_train.py --steps 20 --cpu-steps 0 > gpurun_out/train_t.log 2>&1 && \
timeout -k 10 200 python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --serial >> gpurun_out/train_t.log 2>&1
s=$?; grep -v amdgpu.ids gpurun_out/train_t.log; exit $s
