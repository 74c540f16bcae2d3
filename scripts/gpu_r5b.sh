#!/bin/bash
# Round 5: the tower's waits (awake vs wall time) with 2 and 4 processes sharing the GPU,
# then the round-4 shared-GPU rehearsal of the N = 2 bench WITH the persistent tower
# (gloo, two ranks on one GPU; never a measurement).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python -u scripts/tower_share_stress.py --procs 2 --seconds 30 --wait-us 20000 --out $O/share2.json > $O/share2.log 2>&1 &&
timeout -k 10 300 python -u scripts/tower_share_stress.py --procs 4 --seconds 30 --wait-us 20000 --out $O/share4.json > $O/share4.log 2>&1 &&
AZG_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --sp-games 32 --steps 10 --warmup 3 --train-steps 10 --big-steps 2 --big-train-steps 2 --pente-games 4 --pente-moves 20 > $O/rehearsal.log 2>&1
