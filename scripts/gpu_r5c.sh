#!/bin/bash
# Round 5: the forward tests (tower recovery + breaker), 4 processes sharing the GPU at
# the default 100 ms bound, then the N = 2 shared-GPU rehearsal with the tower on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/tower_share_stress.py --procs 4 --seconds 30 --wait-us 100000 --out $O/share4.json > $O/share4.log 2>&1 &&
AZG_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --sp-games 32 --steps 10 --warmup 3 --train-steps 10 --big-steps 2 --big-train-steps 2 --pente-games 4 --pente-moves 20 > $O/rehearsal.log 2>&1
