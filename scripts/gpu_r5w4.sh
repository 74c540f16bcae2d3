#!/bin/bash
# tower shape 13 (128x64, 4 waves of 64x32, 256 VGPRs; removed after this measurement): forward parity first, then tower timings
set -o pipefail
O=gpurun_out/r5w4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 300 --timeout-method thread > $O/tests_fwd.log 2>&1 &&
timeout -k 10 400 python -u scripts/h3_tune_study.py --batches 512,1024,2048,3456 > $O/study_6x128.jsonl 2> $O/study.err &&
timeout -k 10 300 python -u scripts/h3_tune_study.py --net 10x256 --batches 512 > $O/study_10x256.jsonl 2>> $O/study.err
