#!/bin/bash
# Round 4 lease j: the dgrad's output stored after its BN-partials arrival (late store,
# as the forward): train GPU tests, bitwise vs round 3's library, step time vs round 3's
# library in the same lease, and the step timeline.
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest rc $s"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -4; [ $s -eq 0 ] || exit $s
AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/ref.npz > $O/cmp_ref.log 2>&1 || exit 1
timeout -k 10 300 python scripts/train_lib_compare.py --out /tmp/new.npz > $O/cmp_new.log 2>&1 || exit 1
python scripts/train_lib_compare.py --compare /tmp/ref.npz /tmp/new.npz | tail -2
for i in 1 2; do
  timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "27=0" > $O/probe_new$i.log 2>&1 || exit 1
  AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "27=0" > $O/probe_r3$i.log 2>&1 || exit 1
  echo "new: $(tail -1 $O/probe_new$i.log | cut -c1-120)"; echo "r3:  $(tail -1 $O/probe_r3$i.log | cut -c1-120)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/tr -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $O/tr.log 2>&1
s=$?; echo "trace rc $s"; [ $s -eq 0 ] || exit $s
python scripts/train_trace_segments.py $O/tr/run_kernel_trace.csv
python scripts/train_step_timeline.py $O/tr/run_kernel_trace.csv > $O/timeline.txt
echo done
