#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/spt
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay.py tests/test_native_mcts.py -x -q --timeout 200 --timeout-method thread > gpurun_out/spt/pytest_sp.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/spt/pytest_sp.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u scripts/selfplay_timeline.py 2>&1 | grep -v amdgpu.ids > gpurun_out/spt/timeline5.json
python3 -c "
import json; d=json.load(open('gpurun_out/spt/timeline5.json'))
print({k: d[k] for k in ['wall_s','boards_per_s','gpu_busy_ms','idle_between_ms','host_search_s']})"
