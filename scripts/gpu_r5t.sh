#!/bin/bash
# full GPU suite with split-fp16 train forward + VAR 99 tower, then the default bench
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
