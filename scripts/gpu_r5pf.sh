#!/bin/bash
# split-fp16 tap loop reading both K16 steps' fragments before the MFMAs (the patch in DESIGN §10;
# built into scripts/_ab/libazg_pv_pf.so for this A/B only, not kept) vs the product library
set -o pipefail
O=gpurun_out/r5pf; mkdir -p $O
AZG_PV_LIB=scripts/_ab/libazg_pv_pf.so timeout -k 10 400 python -u scripts/h3_tune_study.py --batches 512,2048,3456 > $O/pf.jsonl 2> $O/study.err &&
timeout -k 10 400 python -u scripts/h3_tune_study.py --batches 512,2048,3456 > $O/base.jsonl 2>> $O/study.err &&
AZG_PV_LIB=scripts/_ab/libazg_pv_pf.so timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 > $O/bt_pf.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 > $O/bt_base.log 2>&1
