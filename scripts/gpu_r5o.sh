#!/bin/bash
# Per-tap fragment addresses (no spills): H3 tile lab + the tower bodies (key 20 = 0 / 1) vs per-layer
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 120 scripts/h3_lab 128 4096 10 > $O/lab_128_4096.jsonl 2>&1 &&
timeout -k 10 120 scripts/h3_lab 256 512 10 > $O/lab_256_512.jsonl 2>&1 &&
timeout -k 10 400 python -u scripts/h3_tune_study.py --vars 0,1 --batches 256,512,1024,2048,3456 > $O/study_6x128.jsonl 2> $O/study_6x128.err &&
timeout -k 10 300 python -u scripts/h3_tune_study.py --vars 0,1 --net 10x256 --batches 256,512 > $O/study_10x256.jsonl 2> $O/study_10x256.err
