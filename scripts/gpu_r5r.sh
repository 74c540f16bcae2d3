#!/bin/bash
# forward GPU tests + a short default bench with the VAR 99 tower
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 300 --timeout-method thread > $O/tests_fwd.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
