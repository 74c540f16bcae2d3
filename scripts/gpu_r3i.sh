#!/bin/bash
# Round 3 lease i: full GPU suite on the rebuilt product library, then the default
# bench line.
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -12; [ $s -le 1 ] || exit $s
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench rc $s"; tail -4 $O/bench.err; [ $s -eq 0 ] || exit $s
echo done
