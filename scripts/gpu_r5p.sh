#!/bin/bash
# h3_tile (pv_h3.h) in the H3 lab
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
timeout -k 10 120 scripts/h3_lab 128 4096 10 > $O/lab_128_4096.jsonl 2>&1 &&
timeout -k 10 120 scripts/h3_lab 128 512 20 > $O/lab_128_512.jsonl 2>&1 &&
timeout -k 10 120 scripts/h3_lab 256 512 10 > $O/lab_256_512.jsonl 2>&1
