#!/bin/bash
# Round 5 final-tree evidence: rocprofv3 kernel traces
# of the headline self-play leg, the configs[1] forward leg and one train run
# -> AZG_TRACE_SCRIPT=gpu_r5f.sh python scripts/summarize_r3.py gpurun_out/r5f gpurun_out/r5f/train/train_trace r5
set -o pipefail
O=gpurun_out/r5f
mkdir -p $O/sp $O/fwd $O/train
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/sp/trace -o run -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0 > $O/sp/bench.json 2> $O/sp/bench.err
s=$?; echo "sp trace rc $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/fwd/trace -o run -- python3 bench.py --steps 20 --warmup 5 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0 > $O/fwd/bench.json 2> $O/fwd/bench.err
s=$?; echo "fwd trace rc $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/train/train_trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/train/train.log 2>&1
s=$?; echo "train trace rc $s"; [ $s -eq 0 ] || exit $s
echo done
