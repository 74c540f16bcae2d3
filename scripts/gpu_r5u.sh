#!/bin/bash
# train forward: fp32 / 3 / 4 split-fp16 products (key 49 = 0 / 1 / 2), then the train tests
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=0 > $O/bt0.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=1 > $O/bt1.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=2 > $O/bt2.log 2>&1 &&
timeout -k 10 1200 python -u -m pytest tests/test_gpu_train.py -v --timeout 900 --timeout-method thread > $O/tests_train.log 2>&1
