#!/bin/bash
# Round 5: weight-grad v2 (slab rows 1 KiB per store) -- bitwise tests, in-process A/B,
# bitwise against round 4's library, kernel traces of both forms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "bitwise or oracle" > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/train_ab.py --variant 48=0 --variant 48=1 --rounds 6 --steps 30 > $O/ab48.log 2>&1 &&
AZG_PV_ALLOW_OLD_ABI=1 AZG_PV_LIB=scripts/_ref/libazg_pv_r4.so timeout -k 10 300 python -u scripts/train_lib_compare.py --out $O/r4.npz > $O/cmp_r4.log 2>&1 &&
timeout -k 10 300 python -u scripts/train_lib_compare.py --out $O/r5.npz > $O/cmp_r5.log 2>&1 &&
timeout -k 10 120 python -u scripts/train_lib_compare.py --compare $O/r4.npz $O/r5.npz > $O/cmp.log 2>&1 &&
rm -f $O/r4.npz $O/r5.npz &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof48_1 -o run -- python3 scripts/bench_train.py --steps 20 --cpu-steps 0 > $O/prof48_1.log 2>&1 &&
find $O/prof48_1 -name "*kernel_stats.csv" -exec cp {} $O/prof48_1_stats.csv \; && rm -rf $O/prof48_1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof48_0 -o run -- python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --tune 48=0 > $O/prof48_0.log 2>&1 &&
find $O/prof48_0 -name "*kernel_stats.csv" -exec cp {} $O/prof48_0_stats.csv \; && rm -rf $O/prof48_0
