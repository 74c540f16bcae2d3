#!/bin/bash
# Round 5, first lease: GPU tests (tower recovery test included), the tower's waits
# alone vs two processes sharing the GPU (scripts/tower_share_stress.py), then the
# default bench without the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 240 python -u scripts/tower_share_stress.py --procs 1 --seconds 20 --wait-us 20000 --out $O/share1.json > $O/share1.log 2>&1 &&
timeout -k 10 300 python -u scripts/tower_share_stress.py --procs 2 --seconds 40 --wait-us 20000 --out $O/share2.json > $O/share2.log 2>&1 &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
