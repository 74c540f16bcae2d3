#!/bin/bash
# train/DP tests + train-step timing + a kernel trace of the train step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_distributed.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/q/pytest.log 2>&1
s=$?; echo "pytest exit $s"; grep -i "flip\|beyond\|passed\|failed\|Error\|assert\|max |dp" gpurun_out/q/pytest.log | grep -v UserWarn | head -60
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 100 python3 scripts/bench_train.py --steps 30 --cpu-steps 0 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/q/trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > gpurun_out/q/trace.log 2>&1
echo "trace exit $?"
