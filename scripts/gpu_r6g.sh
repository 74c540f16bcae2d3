#!/bin/bash
# Round 6: the GPU suite, smoke, the bench, its rocprofv3 kernel-trace summary and the board16
# PMC traffic passes on the key 19 = 2 default (-> gpurun_out/r6g).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
