#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tc
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tc/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/tc/pytest.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 python3 -u scripts/train_ab.py --rounds 4 --steps 20 --variant 12=0 --variant 12=1 2>&1 | grep -v amdgpu.ids
s=$?; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tc/trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > gpurun_out/tc/trace.log 2>&1
echo "trace exit $?"
