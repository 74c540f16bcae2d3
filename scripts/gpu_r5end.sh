#!/bin/bash
# end-of-round check on the committed tree: the full GPU suite, smoke, the default bench
set -o pipefail
O=gpurun_out/r5end; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
