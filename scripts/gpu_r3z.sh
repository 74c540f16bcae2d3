#!/bin/bash
# Round 3 lease z: the final-state evidence of this session -- full GPU suite, smoke(),
# the default bench line, the train-step kernel trace with its segment medians, and the
# train-step A/B of the tail reductions (key 39: 2 default, 1 the side stream).  (A first
# run at commit 64f9dc9 carried the A/B of the stream-K forward, key 44, removed after.)
set -o pipefail
O=gpurun_out/r3z
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke rc $s"; tail -3 $O/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench rc $s"; tail -2 $O/bench.err; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_trace_segments.py $O/tr/run_kernel_trace.csv
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "39=2;39=1;39=2;39=1" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
echo done
