#!/bin/bash
# Round 4 lease o: the C = 256 128x64 tower body with board-keyed halo rows (VAR 33, now
# the product) vs round 3's VAR 32 (study key 10 = 16) across batches, bitwise; the
# 64x64 tile with the same body (key 10 = 14, shape 5); then the forward GPU tests.
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
for b in 128 300 512 1024 2048; do
  for v in 0 16 0 16; do
    AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so timeout -k 10 120 python3 scripts/conv_probe.py --batch $b --tower 1 --tower-shape 8 --var $v --blocks 10 --channels 256 --steps 4 --check 2>/dev/null | tail -1 | cut -c1-230 || exit 1
  done
done
for b in 128 300 512; do
  for v in 0 14; do
    AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so timeout -k 10 120 python3 scripts/conv_probe.py --batch $b --tower 1 --tower-shape 5 --var $v --blocks 10 --channels 256 --steps 4 --check 2>/dev/null | tail -1 | cut -c1-230 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -1 $O/pytest.log; exit $s
