#!/bin/bash
# Round 6: board16 PMC traffic + SQ passes, small-batch latency of the two split arithmetics,
# and the bench under rocprofv3 --kernel-trace --stats (-> gpurun_out/r6h, pmc_b16, r6e16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 300 python -u scripts/small_batch_latency.py > $O/latency.log 2>&1 || exit 1
bash scripts/gpu_pmc_board16.sh > $O/pmc.log 2>&1 || exit 1
bash scripts/gpu_pmc_sq.sh gpurun_out/r6e16 --tower 1 --tower-shape 14 --batch 512 > $O/sq.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
