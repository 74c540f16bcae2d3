#!/bin/bash
# Round 5: forward + train GPU tests (tower recovery / breaker; weight-grad v2 bitwise),
# the weight-grad v2 A/B in-process (bitwise + interleaved timing), the train step bitwise
# against round 4's library, kernel traces of both weight-grad forms, then 4 processes
# sharing the GPU and the N = 2 shared-GPU rehearsal with the tower on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_train.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/train_ab.py --variant 48=0 --variant 48=1 --rounds 6 --steps 30 > $O/ab48.log 2>&1 &&
AZG_PV_LIB=scripts/_ref/libazg_pv_r4.so timeout -k 10 300 python -u scripts/train_lib_compare.py --out $O/r4.npz > $O/cmp_r4.log 2>&1 &&
timeout -k 10 300 python -u scripts/train_lib_compare.py --out $O/r5.npz > $O/cmp_r5.log 2>&1 &&
timeout -k 10 120 python -u scripts/train_lib_compare.py --compare $O/r4.npz $O/r5.npz > $O/cmp.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof48_1 -o run -- python3 scripts/bench_train.py --steps 20 --cpu-steps 0 > $O/prof48_1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof48_0 -o run -- python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --tune 48=0 > $O/prof48_0.log 2>&1 &&
timeout -k 10 300 python -u scripts/tower_share_stress.py --procs 4 --seconds 30 --wait-us 100000 --out $O/share4.json > $O/share4.log 2>&1 &&
AZG_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --sp-games 32 --steps 10 --warmup 3 --train-steps 10 --big-steps 2 --big-train-steps 2 --pente-games 4 --pente-moves 20 > $O/rehearsal.log 2>&1
