#!/bin/bash
# write-through (key 18) A/B of the train step + a serial-mode kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wt
timeout -k 10 300 python3 -u scripts/train_ab.py --rounds 6 --steps 20 --variant 18=0 --variant 18=1 --variant 18=2 \
  --variant 18=4 --variant 18=7 --variant 12=1,18=0 --variant 12=1,18=7 2>&1 | grep -v amdgpu.ids | tee gpurun_out/wt/ab.log
s=$?; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wt/serial -o run -- \
  python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --serial --tune 18=7 > gpurun_out/wt/serial.log 2>&1
s=$?; echo "serial trace exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wt/overlap -o run -- \
  python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --tune 18=7 > gpurun_out/wt/overlap.log 2>&1
echo "overlap trace exit $?"
