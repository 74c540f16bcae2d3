#!/bin/bash
# split-fp16 train forward (key 49): step time A/B, then the train + forward GPU tests
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=0 > $O/bt_49_0.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=1 > $O/bt_49_1.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=0 > $O/bt_49_0b.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=1 > $O/bt_49_1b.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 600 --timeout-method thread > $O/tests_train.log 2>&1 ;
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 300 --timeout-method thread > $O/tests_fwd.log 2>&1
