#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 python -u scripts/h3_bitwise_probe.py > $O/probe.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_forward.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/h3_tune_study.py > $O/study_6x128.log 2>&1 &&
timeout -k 10 300 python -u scripts/h3_tune_study.py --net 10x256 --batches 64,256,512 --rounds 2 --reps 2 > $O/study_10x256.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v -s --timeout 600 --timeout-method thread -k world2 > $O/dist.log 2>&1
