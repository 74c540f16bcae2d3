#!/bin/bash
# Round-2 GPU check: parity tests, smoke, full bench (self-play headline to game end).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
s=$?; echo "pytest gpu exit $s"; tail -5 gpurun_out/pytest_gpu.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -3 gpurun_out/smoke.log
[ $s -eq 0 ] || exit $s
timeout -k 10 ${T_BENCH:-900} python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2> gpurun_out/bench.err
s=$?; echo "bench exit $s"; tail -c 3000 gpurun_out/bench.log; tail -20 gpurun_out/bench.err
exit $s
