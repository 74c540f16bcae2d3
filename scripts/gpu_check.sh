#!/bin/bash
# GPU-box check: parity tests, smoke, short bench.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_status() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash)
timeout -k 10 ${T_TEST:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
s=$?; echo "pytest gpu exit $s"; tail -5 gpurun_out/pytest_gpu.log
ok_status $s || exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -3 gpurun_out/smoke.log
ok_status $s || exit $s
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
s=$?; echo "bench exit $s"; tail -3 gpurun_out/bench.log
exit $s
