#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5k
mkdir -p $O
AZG_TUNE_LOG=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --train-steps 0 --big-steps 0 --pente-moves 0 > $O/bench.json 2> $O/bench.err
