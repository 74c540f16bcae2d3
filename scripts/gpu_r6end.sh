#!/bin/bash
# Round 6 end-of-round evidence on the final tree (-> gpurun_out/r6end): the GPU suite,
# smoke, the default bench line, the bench under rocprofv3 --kernel-trace --stats, the
# board16 SQ and PMC traffic passes.  Every GPU step under its own time limit, chained.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6end
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --sp32-games 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
bash scripts/gpu_pmc_sq.sh $O/sq --tower 1 --tower-shape 14 --batch 512 > $O/sq.log 2>&1 &&
bash scripts/gpu_pmc_board16.sh > $O/pmc.log 2>&1
