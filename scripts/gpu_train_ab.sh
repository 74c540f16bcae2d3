#!/bin/bash
# train-step A/B: gradient tests, then timings for the given tuning variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 200 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 150 --timeout-method thread -k "gradients or trajectory" > gpurun_out/ab/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/ab/pytest.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
for v in "$@"; do
  timeout -k 10 100 python3 scripts/bench_train.py --steps 30 --cpu-steps 0 $v 2>&1 | grep -v amdgpu.ids || exit 1
done
