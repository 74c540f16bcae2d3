#!/bin/bash
# Round 3 lease c: the full default bench line; rocprofv3 kernel traces of the
# configs[2] self-play run and of the configs[1] forward leg; PMC passes for the
# rooflines' traffic (scripts/gpu_pmc_r3.sh); wgrad split-K sweep of the train step.
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O/sp $O/fwd
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench rc $s"; tail -4 $O/bench.err; [ $s -eq 0 ] || exit $s
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/sp/trace -o run -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0 > $O/sp/bench.json 2> $O/sp/bench.err
s=$?; echo "self-play trace rc $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/fwd/trace -o run -- python3 bench.py --steps 20 --warmup 5 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0 > $O/fwd/bench.json 2> $O/fwd/bench.err
s=$?; echo "forward trace rc $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 900 bash scripts/gpu_pmc_r3.sh > $O/pmc.log 2>&1
s=$?; cat $O/pmc.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --splits 0,48,40,32,24,16 --only-splits > $O/splits.log 2>&1
s=$?; tail -2 $O/splits.log; [ $s -eq 0 ] || exit $s
echo done
