#!/bin/bash
# Round 5: the product with split-fp16 eval convs (tower VAR 98, per-layer VAR 99): the whole
# GPU suite, the default bench, then PMC traffic passes of the split-fp16 towers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
OUT=$O/pmc bash scripts/gpu_pmc_r5.sh > $O/pmc.log 2>&1
