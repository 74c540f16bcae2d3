#!/bin/bash
# game-level oracle parity with the exemption gates, incl. the 400-sim to-game-end case
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_oracle_games.py -x -v -s --timeout 900 --timeout-method thread > $O/games.log 2>&1
