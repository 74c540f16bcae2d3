#!/bin/bash
# PMC traffic of the h3_tile towers (shape 12), then the full GPU suite and the default bench
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r5c SHAPE_128=12 SHAPE_256=12 timeout -k 10 600 bash scripts/gpu_pmc_r5.sh > $O/pmc.log 2>&1 &&
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
