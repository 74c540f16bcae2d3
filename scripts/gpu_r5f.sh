#!/bin/bash
# Round 5: split-fp16 (H3) eval tower study -- timing + accuracy against the fp32 tower
# and the fp64 oracle (scripts/tower_h3_ab.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 300 python -u scripts/tower_h3_ab.py --batches 512,3456 > $O/h3_6x128.log 2>&1 &&
timeout -k 10 300 python -u scripts/tower_h3_ab.py --net 10x256 --batches 512 --rounds 3 --reps 3 > $O/h3_10x256.log 2>&1
