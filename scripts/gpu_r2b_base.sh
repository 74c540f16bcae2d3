#!/bin/bash
# Round-2 (session 2) re-baseline: GPU parity tests + overlapped train-step trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/b2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b2/pytest_gpu.log 2>&1
s=$?; echo "pytest gpu exit $s"; tail -3 gpurun_out/b2/pytest_gpu.log
[ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/b2/ov -o run -- \
  python3 scripts/bench_train.py --steps 20 --cpu-steps 0 > gpurun_out/b2/ov.log 2>&1
s=$?; echo "trace exit $s"; tail -5 gpurun_out/b2/ov.log
exit $s
