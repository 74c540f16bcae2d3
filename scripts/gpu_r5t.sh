#!/bin/bash
# self-play headline: the autotuner's tower choices (AZG_TUNE_LOG) vs the h3_tile tower forced (key 5 = 1, key 6 = 12)
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
S="--skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0"
AZG_TUNE_LOG=1 timeout -k 10 300 python -u bench.py $S > $O/auto.log 2> $O/auto.err &&
timeout -k 10 300 python -u bench.py $S --tune 5=1 --tune 6=12 > $O/h3tile.log 2>&1 &&
AZG_TUNE_LOG=1 timeout -k 10 300 python -u bench.py $S > $O/auto2.log 2> $O/auto2.err &&
timeout -k 10 300 python -u bench.py $S --tune 5=1 --tune 6=12 > $O/h3tile2.log 2>&1
