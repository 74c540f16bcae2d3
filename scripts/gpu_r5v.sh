#!/bin/bash
# final round-5 validation: train step, full GPU suite, default bench, N=2 rehearsal, smoke
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 > $O/bt_a.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_train.py --steps 30 --cpu-steps 0 --tune 49=0 > $O/bt_fp32.log 2>&1 &&
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 &&
timeout -k 10 60 echo "rehearsal" > /dev/null &&
AZG_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --sp-games 32 --steps 10 --warmup 3 --train-steps 10 --big-steps 2 --big-train-steps 2 --pente-games 4 --pente-moves 20 > $O/rehearsal.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
