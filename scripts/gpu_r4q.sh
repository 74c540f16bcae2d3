#!/bin/bash
# Round 4 lease q (final tree): the whole GPU suite + smoke, then the default bench line.
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -3; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke rc $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench rc $s"; tail -c 200 $O/bench.err; exit $s
