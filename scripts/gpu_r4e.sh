#!/bin/bash
# Round 4 lease e: the weight-grad launch carrying the previous slab reduction (key 47):
# train GPU tests, bitwise against round 3's library, the step timeline, the A/B.
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -6; [ $s -eq 0 ] || exit $s
AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/ref.npz > $O/cmp_ref.log 2>&1 || exit 1
timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/new.npz > $O/cmp_new.log 2>&1 || exit 1
python scripts/train_lib_compare.py --compare /tmp/ref.npz /tmp/new.npz | tail -4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_trace_segments.py $O/tr/run_kernel_trace.csv
python scripts/train_step_timeline.py $O/tr/run_kernel_trace.csv > $O/timeline.txt
timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "47=1;47=0" > $O/probe.log 2>&1
s=$?; tail -1 $O/probe.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/train_r3_probe.py --only-splits --splits 32,40,48,56 > $O/splits.log 2>&1; s=$?; tail -2 $O/splits.log; [ $s -eq 0 ] || exit $s
echo done
