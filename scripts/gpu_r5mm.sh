#!/bin/bash
# split-fp16 bodies on v_mfma_f32_16x16x32_f16 (AZG_H3_MMA16): tower/per-layer timings, forward + train tests
set -o pipefail
O=gpurun_out/r5mm; mkdir -p $O
timeout -k 10 400 python -u scripts/h3_tune_study.py --batches 512,1024,2048,3456 > $O/study_6x128.jsonl 2> $O/study.err &&
timeout -k 10 300 python -u scripts/h3_tune_study.py --net 10x256 --batches 512 > $O/study_10x256.jsonl 2>> $O/study.err &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 300 --timeout-method thread > $O/tests_fwd.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 > $O/bt.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 600 --timeout-method thread > $O/tests_train.log 2>&1
